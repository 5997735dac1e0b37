#!/usr/bin/env bash
# One parametrised runner for the GPU box (replaces the round-5 one-off wrappers gpu_r5_*.sh / ab_*.sh).
# usage (via gpurun):  bash tools/gpu.sh TASK TAG [ARGS...]
#   suite TAG [PYTEST_K]    the -m gpu suite (optionally -k PYTEST_K) + smoke; parity reports -> gpurun_out/parity_reports_TAG.jsonl
#   tests TAG FILE_OR_K     one test file / node id / -k expression of the gpu suite
#   bench TAG [ARGS...]     bench.py [ARGS] -> gpurun_out/bench_TAG.json (+ .err)
#   prof TAG                rocprofv3 kernel trace + stats of the default bench command (tools/prof_default_bench.sh)
#   pmc TAG                 FETCH_SIZE / WRITE_SIZE passes per precision (tools/gpu_profile.sh, SKIP_KT=1)
#   n2 TAG                  `python bench.py --gpus 2` (no launcher: bench.py starts its ranks) with two gloo ranks on one card
#   pg1 TAG                 the N-rank schedule at world 1 over RCCL vs the plain N=1 line (tools/rehearse_pg_world1.sh)
#   py TAG SCRIPT [ARGS]    python SCRIPT ARGS -> gpurun_out/py_TAG.log
# Every GPU step runs under its own timeout and the steps stop at the first failure.
set -u
TASK=${1:?task}
TAG=${2:?tag}
shift 2
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
case "$TASK" in
  suite)
    rm -f gpurun_out/parity_reports.jsonl
    K=()
    [ $# -ge 1 ] && K=(-k "$1")
    timeout -k 10 1100 $PYT tests -m gpu "${K[@]}" > gpurun_out/gpu_tests_$TAG.log 2>&1
    rc=$?
    cp gpurun_out/parity_reports.jsonl gpurun_out/parity_reports_$TAG.jsonl 2>/dev/null
    [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 ;;
  tests)
    rm -f gpurun_out/parity_reports.jsonl
    timeout -k 10 1100 $PYT -m gpu "$@" > gpurun_out/gpu_tests_$TAG.log 2>&1
    rc=$?
    cp gpurun_out/parity_reports.jsonl gpurun_out/parity_reports_$TAG.jsonl 2>/dev/null
    exit $rc ;;
  bench)
    timeout -k 10 900 python bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err ;;
  prof)
    bash tools/prof_default_bench.sh "$TAG" ;;
  pmc)
    SKIP_KT=1 bash tools/gpu_profile.sh "$TAG" ;;
  n2)
    YANERF_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 5 --warmup 2 "$@" \
      > gpurun_out/bench_$TAG.raw 2> gpurun_out/bench_$TAG.err && grep "^{" gpurun_out/bench_$TAG.raw > gpurun_out/bench_$TAG.json ;;
  pg1)
    bash tools/rehearse_pg_world1.sh "$TAG" ;;
  py)
    S=${1:?script}
    shift
    timeout -k 10 900 python -u "$S" "$@" > gpurun_out/py_$TAG.log 2>&1 ;;
  *)
    echo "unknown task $TASK" >&2
    exit 2 ;;
esac
