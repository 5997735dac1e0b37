# round 5: the bf16 Lego step (bench.py headline window, --precision bf16) with MFMA padding variants vs the in-tree build,
# interleaved three times; one JSON line per run into gpurun_out/pad_bench.jsonl
set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
: > gpurun_out/pad_bench.jsonl
for r in 1 2 3; do
  for L in in-tree build/var_pad50.so build/var_pad25.so; do
    if [ "$L" = in-tree ]; then
      v=$(timeout -k 10 300 python bench.py --precision bf16 --steps 40 --warmup 5 --no-extras --psnr-steps 0 --no-cpu-baseline --secondary none 2>/dev/null) || exit $?
    else
      v=$(YANERF_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 300 python bench.py --precision bf16 --steps 40 --warmup 5 --no-extras --psnr-steps 0 --no-cpu-baseline --secondary none 2>/dev/null) || exit $?
    fi
    echo "{\"lib\": \"$L\", \"round\": $r, \"r\": $v}" >> gpurun_out/pad_bench.jsonl
  done
done
