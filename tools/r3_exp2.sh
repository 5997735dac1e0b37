#!/usr/bin/env bash
# A/B of variant libraries against the in-tree build (MLP microbench, two interleaved rounds) + fp32 dW HBM traffic of
# the XCD-paired k-tiles. usage (via gpurun): bash tools/r3_exp2.sh TAG
set -u
TAG=${1:-x2}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out"
bash tools/ab_libs.sh ${TAG}_bf16 bf16 build/abl256.so build/pp_inphase.so || exit $?
bash tools/ab_libs.sh ${TAG}_fp32 fp32,fp32x3 build/xpair.so || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
  YANERF_HIP_LIB=$GRAFT_REPO_ROOT/build/xpair.so timeout -k 10 120 rocprofv3 --pmc $C -d "$OUT/${TAG}_xpair_$C" -o run --output-format csv -- python tools/microbench.py fp32 > "$OUT/${TAG}_xpair_$C.log" 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --pmc $C -d "$OUT/${TAG}_base_$C" -o run --output-format csv -- python tools/microbench.py fp32 > "$OUT/${TAG}_base_$C.log" 2>&1 || exit $?
done
python tools/pmc_summary.py "$OUT/${TAG}_xpair_FETCH_SIZE" "$OUT/${TAG}_xpair_WRITE_SIZE" mlp_dw_kernel "$OUT/${TAG}_pmc_dw_xpair.json" > /dev/null 2>&1
python tools/pmc_summary.py "$OUT/${TAG}_base_FETCH_SIZE" "$OUT/${TAG}_base_WRITE_SIZE" mlp_dw_kernel "$OUT/${TAG}_pmc_dw_base.json" > /dev/null 2>&1
