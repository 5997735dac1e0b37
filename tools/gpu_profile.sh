#!/usr/bin/env bash
# Profiles for profiles/: (1) rocprofv3 kernel-trace stats of the default bench command, (2) HBM traffic of the
# MLP kernels from separate FETCH_SIZE / WRITE_SIZE passes (never combined with trace domains), per precision.
# usage (via gpurun): [SKIP_KT=1] bash tools/gpu_profile.sh TAG   (SKIP_KT: PMC passes only)
set -u
TAG=${1:-prof}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out"
[ -n "${SKIP_KT:-}" ] || timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_kt" -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --psnr-steps 0 > "$OUT/${TAG}_kt.log" 2>&1 || exit $?
for P in fp32 bf16 fp32x3 bf16s; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $C -d "$OUT/${TAG}_${P}_$C" -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras --psnr-steps 0 --secondary none --precision $P > "$OUT/${TAG}_${P}_$C.log" 2>&1 || exit $?
  done
  for K in mlp_fwd_kernel mlp_bwd_dx_kernel mlp_dw_kernel; do
    python tools/pmc_summary.py "$OUT/${TAG}_${P}_FETCH_SIZE" "$OUT/${TAG}_${P}_WRITE_SIZE" $K "$OUT/${TAG}_pmc_${K}_${P}.json" >> "$OUT/${TAG}_pmc.log" 2>&1 || exit $?
  done
done
