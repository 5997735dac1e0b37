#!/usr/bin/env bash
# Round-4 A/B of the bf16 dW point-split count: the MLP microbench at the Lego fine pass under each split count
# (the A/B build read it from YANERF_AB_SPLITS_PM; results in profiles/r4_ab_bf16_dw_splits.jsonl). Kept as the record
# of how that file was made; the shipped library ignores the variable.
set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
: > gpurun_out/ab_splits.jsonl
for r in 1 2; do
  for S in 32 18 36 16 24 28; do
    echo "{\"S\": $S, \"round\": $r, \"res\": $(YANERF_AB_SPLITS_PM=$S timeout -k 10 200 python tools/microbench.py bf16 2>/dev/null)}" >> gpurun_out/ab_splits.jsonl || exit $?
  done
done
