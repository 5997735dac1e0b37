#!/usr/bin/env bash
# rocprofv3 kernel trace + stats of the DEFAULT bench command (what the driver runs), with the per-launch-shape
# summary that the bench's roofline kernel timing is compared against.
# usage (via gpurun): bash tools/prof_default_bench.sh TAG
set -u
TAG=${1:-pd}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_kt" -o run --output-format csv -- python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
python tools/kstats_by_launch.py gpurun_out/${TAG}_kt gpurun_out/${TAG}_by_launch.json > gpurun_out/${TAG}_by_launch.txt
rm -f gpurun_out/${TAG}_kt/*/run_kernel_trace.csv gpurun_out/${TAG}_kt/run_kernel_trace.csv 2>/dev/null || true
