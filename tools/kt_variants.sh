#!/usr/bin/env bash
# Per-kernel times (rocprofv3 kernel stats of the MLP microbench) for prebuilt variant libraries.
# usage (via gpurun): bash tools/kt_variants.sh TAG PREC lib1.so lib2.so ...   ("base" = the in-tree build)
set -u
TAG=$1; PREC=$2; shift 2
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
for LIB in "$@"; do
  NAME=$(basename $LIB .so)
  if [ "$LIB" = base ]; then unset YANERF_HIP_LIB; else export YANERF_HIP_LIB=$GRAFT_REPO_ROOT/$LIB; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/ktv_${TAG}_$NAME" -o run --output-format csv -- python tools/microbench.py $PREC > gpurun_out/ktv_${TAG}_$NAME.log 2>&1 || exit $?
  echo "== $NAME" >> gpurun_out/ktv_$TAG.txt
  python tools/kstats.py gpurun_out/ktv_${TAG}_$NAME 6 >> gpurun_out/ktv_$TAG.txt
done
