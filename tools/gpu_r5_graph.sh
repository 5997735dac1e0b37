set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "graph" > gpurun_out/gpu3_tests.log 2>&1 || exit $?
for K in 1 4 8; do timeout -k 10 200 python tools/fern_steps.py bf16 32 graph $K > gpurun_out/fern3_graph_$K.txt 2>&1 || exit $?; done
timeout -k 10 200 python tools/fern_steps.py bf16 32 eager > gpurun_out/fern3_eager.txt 2>&1 || exit $?
bash tools/ab_libs.sh wg1 bf16 build/var_wg1.so
for r in 1 2; do for ov in serial early both split; do timeout -k 10 200 python tools/fern_steps.py bf16 40 eager 1 $ov >> gpurun_out/fern3_sched.txt 2>&1 || exit $?; done; done
