#!/usr/bin/env bash
# L2 (TCC) counter passes over the MLP microbench: hit/miss and memory-side request counts per kernel, to see
# whether a kernel's weights stay L2-resident (one pass per counter group, no trace domains beside --pmc).
set -u
TAG=${1:-tcc}
PREC=${2:-fp32,bf16,fp32x3}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_p1" -o run --output-format csv -- python tools/microbench.py $PREC > gpurun_out/${TAG}_p1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_p2" -o run --output-format csv -- python tools/microbench.py $PREC > gpurun_out/${TAG}_p2.log 2>&1 || exit $?
python tools/sq_summary.py gpurun_out/${TAG}_summary.json gpurun_out/${TAG}_p1 gpurun_out/${TAG}_p2 > /dev/null
