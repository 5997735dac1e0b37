set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/mo
export TMPDIR=/tmp
python tools/mfma_order_model.py gen f32 2000 gpurun_out/mo/f32.bin && python tools/mfma_order_model.py gen bf16 2000 gpurun_out/mo/bf16.bin
timeout -k 10 60 tools/probes/probe_mfma_order gpurun_out/mo/f32.bin gpurun_out/mo/f32.out && \
timeout -k 10 60 tools/probes/probe_mfma_order gpurun_out/mo/bf16.bin gpurun_out/mo/bf16.out && \
rm -f gpurun_out/mo/*.bin gpurun_out/mo/*.npz && \
YANERF_PARITY_DUMP=gpurun_out/parity_dump timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "test_render_eval_lego or test_trainer_render_matches_reference_render or test_fern_render_with_tensor_bounds" > gpurun_out/gpu1_tests.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "test_backward_schedules_give_identical_steps or test_bucketed_and_single_exchange or test_trainer_gradient_exchange_two_ranks or test_graph_render" > gpurun_out/gpu1b_tests.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "test_trainer_trajectory" > gpurun_out/gpu1c_tests.log 2>&1
for s in 42 1 7; do timeout -k 10 300 python tools/psnr_synthetic.py --size 50 --rays 1024 --steps 1000 --seed $s --precisions fp32 > gpurun_out/collapse_ours_s$s.json 2>&1 || exit 1; done
