#!/bin/bash
# GPU box: bench.py under each environment setting given as one quoted string (e.g. "RT_TRACE_GRID_PCT=90"),
# alternating REPS times (default 2), for the bench.py arguments in ARGS (default "--config c3").
# Prints one line per run: setting, Mrays/s, ms per frame.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/env
for rep in $(seq 1 ${REPS:-2}); do
  k=0
  for setting in "$@"; do
    k=$((k + 1))
    log=gpurun_out/env/${k}_${rep}.log
    env $setting timeout -k 10 300 python bench.py ${ARGS:---config c3} --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline \
        --c4-steps 0 > $log 2>&1 || { echo "[$setting] failed"; tail -5 $log; exit 1; }
    echo "[$setting] $(tail -1 $log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
