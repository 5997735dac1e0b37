# round 5: configs_at_n over RCCL at world 1 vs no process group, interleaved twice
set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
: > gpurun_out/cfgn_world1.jsonl
for r in 1 2; do for m in plain pg; do
  timeout -k 10 300 python tools/rehearse_configs_at_n_world1.py $m >> gpurun_out/cfgn_world1.jsonl 2> gpurun_out/cfgn_$m.err || exit $?
done; done
