set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/gpu_r5_mall.sh || exit $?
bash tools/round_check.sh ${1:-r5b} || exit $?
