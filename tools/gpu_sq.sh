#!/usr/bin/env bash
# SQ counter passes (then FETCH_SIZE / WRITE_SIZE) over the MLP microbench (no trace domains beside --pmc; one pass per counter group).
set -u
TAG=${1:-sq}; PREC=${2:-fp32,bf16,fp32x3}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_p1" -o run --output-format csv -- python tools/microbench.py $PREC > gpurun_out/${TAG}_p1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_p2" -o run --output-format csv -- python tools/microbench.py $PREC > gpurun_out/${TAG}_p2.log 2>&1 || exit $?
true
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_$C" -o run --output-format csv -- python tools/microbench.py $PREC > gpurun_out/${TAG}_$C.log 2>&1 || exit $?
done
python tools/sq_summary.py gpurun_out/${TAG}_summary.json gpurun_out/${TAG}_p1 gpurun_out/${TAG}_p2 gpurun_out/${TAG}_FETCH_SIZE gpurun_out/${TAG}_WRITE_SIZE > /dev/null
