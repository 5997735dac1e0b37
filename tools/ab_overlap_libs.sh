#!/usr/bin/env bash
# tools/ab_overlap.py (the fused step under each backward schedule) for the in-tree library and each variant library.
# usage (via gpurun): bash tools/ab_overlap_libs.sh TAG PREC build/a.so ...
set -u
TAG=$1; PREC=$2; shift 2
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
OUT=gpurun_out/abov_$TAG.jsonl
: > $OUT
echo "{\"lib\": \"in-tree\", \"r\": $(timeout -k 10 300 python tools/ab_overlap.py $PREC 2>/dev/null)}" >> $OUT || exit $?
for L in "$@"; do
  echo "{\"lib\": \"$L\", \"r\": $(YANERF_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 300 python tools/ab_overlap.py $PREC 2>/dev/null)}" >> $OUT || exit $?
done
