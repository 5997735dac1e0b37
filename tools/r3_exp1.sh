#!/usr/bin/env bash
# Round-3 experiments, then the round evidence: (1) f32 MFMA + VALU co-issue probe, (2) bf16 weight-stream ablation
# (YANERF_ABLATE=256: every weight fragment from K-block 0), (3) fp32 dW k-tiles of a split on one XCD
# (YANERF_DW_XPAIR=1) timing + HBM traffic, (4) tools/round_evidence.sh.
# usage (via gpurun): bash tools/r3_exp1.sh TAG
set -u
TAG=${1:-x1}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 60 ./tools/probes/probe_mfma_valu > $OUT/${TAG}_probe_mfma_valu.jsonl 2>&1 || exit $?
bash tools/ab_libs.sh ${TAG}_abl256 bf16 build/abl256.so || exit $?
bash tools/ab_libs.sh ${TAG}_xpair fp32,fp32x3 build/xpair.so || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
  YANERF_HIP_LIB=$GRAFT_REPO_ROOT/build/xpair.so timeout -k 10 120 rocprofv3 --pmc $C -d "$OUT/${TAG}_xpair_$C" -o run --output-format csv -- python tools/microbench.py fp32 > "$OUT/${TAG}_xpair_$C.log" 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --pmc $C -d "$OUT/${TAG}_base_$C" -o run --output-format csv -- python tools/microbench.py fp32 > "$OUT/${TAG}_base_$C.log" 2>&1 || exit $?
done
python tools/pmc_summary.py "$OUT/${TAG}_xpair_FETCH_SIZE" "$OUT/${TAG}_xpair_WRITE_SIZE" mlp_dw_kernel "$OUT/${TAG}_pmc_dw_xpair.json" > /dev/null 2>&1
python tools/pmc_summary.py "$OUT/${TAG}_base_FETCH_SIZE" "$OUT/${TAG}_base_WRITE_SIZE" mlp_dw_kernel "$OUT/${TAG}_pmc_dw_base.json" > /dev/null 2>&1
bash tools/round_evidence.sh ${TAG}
