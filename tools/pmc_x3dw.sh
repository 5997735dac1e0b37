#!/usr/bin/env bash
# SQ counters of the MLP kernels under tools/microbench.py for each given library (in-tree first), one PMC pass each
# (no trace domains), summarised per kernel by tools/sq_summary.py into gpurun_out/pmc_TAG_<n>.json.
# usage (via gpurun): bash tools/pmc_x3dw.sh TAG PREC [build/a.so ...]
set -u
TAG=$1; PREC=$2; shift 2
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY"
n=0
for L in in-tree "$@"; do
  if [ "$L" = in-tree ]; then unset YANERF_HIP_LIB; else export YANERF_HIP_LIB=$GRAFT_REPO_ROOT/$L; fi
  timeout -s KILL 120 rocprofv3 --pmc $C -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_${TAG}_$n" -o run --output-format csv -- python tools/microbench.py $PREC > gpurun_out/pmc_${TAG}_$n.log 2>&1 || exit $?
  python tools/sq_summary.py gpurun_out/pmc_${TAG}_$n.json gpurun_out/pmc_${TAG}_$n > /dev/null || exit $?
  echo "$n $L" >> gpurun_out/pmc_${TAG}_libs.txt
  n=$((n + 1))
done
