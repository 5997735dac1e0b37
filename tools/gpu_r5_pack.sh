# round 5: one pack launch for both models, and the pack beside the ray generation -- tests, Fern A/B, bench
set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer.py -x -v --timeout 120 --timeout-method thread \
  -k "pack_multi or graph or trajectory or schedules or lr_schedule or registry_step" \
  > gpurun_out/pack_tests.log 2>&1 || exit $?
: > gpurun_out/pack_fern.txt
for r in 1 2 3; do
  timeout -k 10 200 python tools/fern_steps.py bf16 80 eager 1 default >> gpurun_out/pack_fern.txt 2>&1 || exit $?
  timeout -k 10 200 python tools/fern_steps.py bf16 80 eager 1 default packside >> gpurun_out/pack_fern.txt 2>&1 || exit $?
  timeout -k 10 200 python tools/fern_steps.py bf16 80 graph 4 default >> gpurun_out/pack_fern.txt 2>&1 || exit $?
  timeout -k 10 200 python tools/fern_steps.py bf16 80 graph 4 default packside >> gpurun_out/pack_fern.txt 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pack_kt -- python tools/fern_steps.py bf16 15 eager 1 default packside \
  > gpurun_out/pack_kt.log 2>&1 || exit $?
python tools/step_timeline.py gpurun_out/pack_kt 3 > gpurun_out/pack_timeline.txt 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_pack.json 2> gpurun_out/bench_pack.err || exit $?
