#!/bin/bash
# GPU box: bench lines for a list of argument sets, alternating twice.
#   bash tools/gpu_sweep2.sh "--shard-of 8 --pool 2097152" "ENV:RT_PARTITIONS=3 --shard-of 8" ...
# An entry starting with ENV:X=Y sets that environment variable for the run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/sweep2
for rep in 1 2; do
  i=0
  for a in "$@"; do
    i=$((i+1))
    envs=""; args="$a"
    while [[ "$args" == ENV:* ]]; do e="${args%% *}"; envs="$envs ${e#ENV:}"; args="${args#* }"; [ "$args" == "$e" ] && args=""; done
    env $envs timeout -k 10 240 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline $args \
        > gpurun_out/sweep2/r${rep}_$i.log 2>&1 || { echo "[$a] failed"; tail -5 gpurun_out/sweep2/r${rep}_$i.log; exit 1; }
    echo "[$a] $(tail -1 gpurun_out/sweep2/r${rep}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
