set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/mall_probe.py bf16 > gpurun_out/mall_intree.json 2> gpurun_out/mall_intree.err || exit $?
YANERF_HIP_LIB=$GRAFT_REPO_ROOT/build/var_aux0.so timeout -k 10 300 python tools/mall_probe.py bf16 > gpurun_out/mall_aux0.json 2> gpurun_out/mall_aux0.err || exit $?
