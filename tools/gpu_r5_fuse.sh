# round 5: one pack launch for both models + Adam with the step advance folded in -- tests, Fern timing, trace, bench
set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer.py -x -v --timeout 120 --timeout-method thread \
  -k "fused_adam or pack_multi or graph or trajectory or schedules or lr_schedule or registry_step" \
  > gpurun_out/fuse_tests.log 2>&1 || exit $?
: > gpurun_out/fuse_fern.txt
for r in 1 2; do
  timeout -k 10 200 python tools/fern_steps.py bf16 60 eager 1 >> gpurun_out/fuse_fern.txt 2>&1 || exit $?
  timeout -k 10 200 python tools/fern_steps.py bf16 60 graph 4 >> gpurun_out/fuse_fern.txt 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fuse_kt -- python tools/fern_steps.py bf16 15 eager 1 \
  > gpurun_out/fuse_kt.log 2>&1 || exit $?
python tools/step_timeline.py gpurun_out/fuse_kt 3 > gpurun_out/fuse_timeline.txt 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_fuse.json 2> gpurun_out/bench_fuse.err || exit $?
