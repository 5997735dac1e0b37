#!/usr/bin/env bash
# round-5: full GPU suite + smoke (parity reports + dumps), x3 coarse dumps, Fern small-batch timelines
set -u
TAG=${1:-r5a}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/parity_reports.jsonl
timeout -k 10 250 python tools/dump_coarse_stage.py fp32x3 > gpurun_out/dump_coarse_x3.log 2>&1 || exit $?
YANERF_PARITY_DUMP=gpurun_out/parity_dump timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
cp gpurun_out/parity_reports.jsonl gpurun_out/parity_reports_$TAG.jsonl 2>/dev/null
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
for m in eager graph; do
  timeout -k 10 200 python tools/fern_steps.py bf16 30 $m > gpurun_out/fern_bf16_$m.txt 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/fern_kt_$m" -o run --output-format csv -- python tools/fern_steps.py bf16 15 $m > gpurun_out/fern_kt_$m.txt 2>&1 || exit $?
  python tools/step_timeline.py gpurun_out/fern_kt_$m 3 gpurun_out/fern_timeline_$m.json > gpurun_out/fern_timeline_$m.txt
  rm -rf gpurun_out/fern_kt_$m
done
exit $rc
