#!/usr/bin/env bash
# round-5 diagnostics: coarse-stage dumps (fp32) and Fern small-batch kernel timelines (bf16 eager / graph)
set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 250 python tools/dump_coarse_stage.py fp32 > gpurun_out/dump_coarse.log 2>&1 || exit $?
for m in eager graph; do
  timeout -k 10 200 python tools/fern_steps.py bf16 30 $m > gpurun_out/fern_bf16_$m.txt 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/fern_kt_$m" -o run --output-format csv -- python tools/fern_steps.py bf16 15 $m > gpurun_out/fern_kt_$m.txt 2>&1 || exit $?
  python tools/step_timeline.py gpurun_out/fern_kt_$m 3 gpurun_out/fern_timeline_$m.json > gpurun_out/fern_timeline_$m.txt
done
