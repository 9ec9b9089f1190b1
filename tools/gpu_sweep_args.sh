#!/bin/bash
# GPU box: bench.py once per "ENV=... -- bench args" setting, alternating REPS times (default 2).
#   tools/gpu_sweep_args.sh "RT_PARTITIONS=2 -- --config c3 --shard-of 8" " -- --config c3 --shard-of 8"
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/sweep
for rep in $(seq 1 ${REPS:-2}); do
  i=0
  for spec in "$@"; do
    i=$((i + 1))
    envs=${spec%%--*}; args=${spec#*-- }
    log=gpurun_out/sweep/s${i}_$rep.log
    env $envs timeout -k 10 300 python bench.py $args --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --c4-steps 0 \
        > $log 2>&1 || { echo "[$spec] failed"; tail -5 $log; exit 1; }
    echo "[$spec] $(tail -1 $log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
