set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
: > gpurun_out/prio_fern.txt
for r in 1 2; do for p in none hiprio; do
  timeout -k 10 200 python tools/fern_steps.py bf16 60 eager 1 default $p >> gpurun_out/prio_fern.txt 2>&1 || exit $?
  timeout -k 10 200 python tools/fern_steps.py bf16 60 eager 1 serial $p >> gpurun_out/prio_fern.txt 2>&1 || exit $?
done; done
timeout -k 10 400 python tools/prio_ab.py bf16 3 > gpurun_out/prio_ab2.json 2> gpurun_out/prio_ab2.err || exit $?
