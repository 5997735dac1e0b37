#!/usr/bin/env bash
# Run a subset of GPU tests (arguments = pytest selectors) plus the Adam emulation probe and smoke.
# usage (via gpurun): bash tools/gpu_newtests.sh TAG tests/test_gpu_trainer.py ...
set -u
TAG=${1:-nt}; shift || true
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/adam_emulation_check.py cuda > gpurun_out/adam_emul_$TAG.json 2> gpurun_out/adam_emul_$TAG.err || exit $?
timeout -k 10 900 python -u -m pytest "$@" -m gpu -v -s -rf --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_$TAG.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
exit $rc
