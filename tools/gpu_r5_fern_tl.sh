# round 5: kernel timeline of the Fern bf16 eager step on the final build
set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fern_final_kt -- python tools/fern_steps.py bf16 15 eager 1 \
  > gpurun_out/fern_final_kt.log 2>&1 || exit $?
python tools/step_timeline.py gpurun_out/fern_final_kt 3 > gpurun_out/fern_final_timeline.txt 2>&1 || exit $?
