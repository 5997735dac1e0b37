set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/parity_reports.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "render_eval_lego or trainer_render_matches or fern_render_with or scatter or graph" > gpurun_out/gpu2_tests.log 2>&1 || exit $?
cp gpurun_out/parity_reports.jsonl gpurun_out/parity_reports_gpu2.jsonl
for m in eager graph; do timeout -k 10 200 python tools/fern_steps.py bf16 30 $m > gpurun_out/fern2_bf16_$m.txt 2>&1 || exit $?; done
bash tools/rehearse_pg_world1.sh pg1
