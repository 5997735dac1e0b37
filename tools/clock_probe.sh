#!/usr/bin/env bash
# Effective shader clock of each MLP kernel: GRBM_GUI_ACTIVE / GRBM_COUNT (GPU-busy cycles, summed over the XCDs) and
# SQ_BUSY_CYCLES per dispatch, with the dispatch durations from the same rocprofv3 run (--pmc with --kernel-trace only).
# usage (via gpurun): bash tools/clock_probe.sh TAG PREC
set -u
TAG=${1:-clk}; PREC=${2:-fp32}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
  -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc" -o run --output-format csv -- python tools/microbench.py $PREC \
  > gpurun_out/${TAG}_pmc.log 2>&1 || exit $?
python tools/clock_summary.py gpurun_out/${TAG}_pmc > gpurun_out/${TAG}_clock.json
