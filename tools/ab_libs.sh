#!/usr/bin/env bash
# MLP microbench of the in-tree library and each given variant library, two interleaved rounds; one JSON line per run
# into gpurun_out/ablibs_TAG.jsonl.
# usage (via gpurun): bash tools/ab_libs.sh TAG PREC build/a.so build/b.so ...
set -u
TAG=$1; PREC=$2; shift 2
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/ablibs_$TAG.jsonl
: > $OUT
for round in 1 2; do
  echo "{\"lib\": \"in-tree\", \"round\": $round, \"r\": $(timeout -k 10 200 python tools/microbench.py $PREC 2>/dev/null)}" >> $OUT || exit $?
  for L in "$@"; do
    echo "{\"lib\": \"$L\", \"round\": $round, \"r\": $(YANERF_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python tools/microbench.py $PREC 2>/dev/null)}" >> $OUT || exit $?
  done
done
