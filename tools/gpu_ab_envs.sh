#!/bin/bash
# GPU box: bench.py A/B over environment settings (read at rt_scene_upload), alternating REPS rounds
# (default 2) over the argument sets in ARGSETS (';'-separated; default: C3, C4, rank 0's share of 8).
#   tools/gpu_ab_envs.sh "" "RT_DRAIN_EVERY=2" "RT_DRAIN_EVERY=3"      ("" = as built)
# One line per run: setting, argument set, Mrays/s, ms per frame.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/abe
IFS=';' read -r -a SETS <<< "${ARGSETS:---config c3;--config c4;--shard-of 8}"
for rep in $(seq 1 ${REPS:-2}); do
  k=0
  for args in "${SETS[@]}"; do
    k=$((k + 1))
    j=0
    for v in "$@"; do
      j=$((j + 1))
      log=gpurun_out/abe/${j}_${k}_${rep}.log
      env $v timeout -k 10 300 python bench.py $args --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --c4-steps 0 \
          > $log 2>&1 || { echo "[$v] [$args] failed"; tail -5 $log; exit 1; }
      echo "[$v] [$args] $(tail -1 $log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    done
  done
done
