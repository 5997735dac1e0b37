# round 5: LLVM AMDGPU scheduler strategies (-mllvm -amdgpu-sched-strategy=...) as variant libraries, bf16 and fp32
set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/ab_libs.sh sched_bf16 bf16 build/var_sched_max-ilp.so build/var_sched_max-memory-clause.so build/var_sched_iterative-ilp.so || exit $?
bash tools/ab_libs.sh sched_fp32 fp32 build/var_sched_max-ilp.so build/var_sched_max-memory-clause.so build/var_sched_iterative-ilp.so || exit $?
