#!/usr/bin/env bash
# GPU test suite (+ smoke) only; parity reports land in gpurun_out/parity_reports.jsonl.
# usage (via gpurun): bash tools/gpu_tests.sh TAG [pytest -k expression]
set -u
TAG=${1:-t}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/parity_reports.jsonl
K=()
if [ $# -ge 2 ]; then K=(-k "$2"); fi
timeout -k 10 900 python -u -m pytest tests -m gpu ${PYX--x} -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  "${K[@]}" > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
