# round 5: the forward's setprio around its bf16 K loop -- microbench A/B against the previous build, bf16 GPU tests, bench
set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_libs.sh prio2 bf16 build/var_head.so || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "bf16" > gpurun_out/prio2_tests.log 2>&1 || exit $?
timeout -k 10 900 python bench.py --no-extras --psnr-steps 0 --no-cpu-baseline > gpurun_out/bench_prio2.json 2> gpurun_out/bench_prio2.err || exit $?
