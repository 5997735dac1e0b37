#!/usr/bin/env bash
# Kernel trace of a short single-precision bench run and the timeline of one training step (tools/step_timeline.py).
# usage (via gpurun): bash tools/timeline.sh TAG PREC
set -u
TAG=${1:-tl}; PREC=${2:-bf16}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_kt" -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --psnr-steps 0 --secondary none --precision $PREC > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
python tools/step_timeline.py gpurun_out/${TAG}_kt ${BACK:-3} gpurun_out/${TAG}_timeline.json > gpurun_out/${TAG}_timeline.txt
gzip -f gpurun_out/${TAG}_kt/run_kernel_trace.csv 2>/dev/null || true
