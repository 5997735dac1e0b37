#!/usr/bin/env bash
# Round-4 A/B of the fp32 / x3 dW point-split count (an A/B build read YANERF_AB_SPLITS; results in
# profiles/r4_ab_fp32_dw_splits.jsonl: 64 = five whole CU rounds stays fastest). The shipped library ignores it.
set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
: > gpurun_out/ab_splits32.jsonl
for r in 1 2; do
  for S in 64 51 77 96 128; do
    echo "{\"S\": $S, \"round\": $r, \"res\": $(YANERF_AB_SPLITS=$S timeout -k 10 200 python tools/microbench.py fp32,fp32x3 2>/dev/null)}" >> gpurun_out/ab_splits32.jsonl || exit $?
  done
done
