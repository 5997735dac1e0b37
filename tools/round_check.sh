#!/usr/bin/env bash
# Full GPU test suite then the default bench command (as the driver runs them at round end).
# usage (via gpurun): bash tools/round_check.sh TAG
set -u
TAG=${1:-rc}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
start=$(date +%s)
timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
echo "bench wall seconds: $(( $(date +%s) - start ))" >> gpurun_out/bench_$TAG.err
