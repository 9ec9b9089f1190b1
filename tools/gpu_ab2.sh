#!/bin/bash
# GPU box: A/B of (library variant, environment) pairs over bench argument sets, alternating REPS times.
#   SPECS="default| head|variant=head p3|RT_PARTITIONS=3" tools/gpu_ab2.sh "--config c3" "--config c4"
# A spec is label|settings, settings space-separated: variant=<name> picks lib/variants/<name>, the
# rest are environment assignments.  Prints one line per run: label, argument set, Mrays/s, ms per frame.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
for rep in $(seq 1 ${REPS:-2}); do
  k=0
  for args in "$@"; do
    k=$((k + 1))
    for spec in $SPECS; do
      label=${spec%%|*}; settings=${spec#*|}
      lib=$PWD/buas-pathtracer_amd/lib/librt_mi355x.so; envs=()
      for kv in ${settings//,/ }; do
        case $kv in variant=*) lib=$PWD/buas-pathtracer_amd/lib/variants/${kv#variant=}/librt_mi355x.so;; *=*) envs+=("$kv");; esac
      done
      log=gpurun_out/ab/${label}_${k}_${rep}.log
      env "${envs[@]}" RT_MI355X_LIB=$lib timeout -k 10 300 python bench.py $args --steps ${STEPS:-5} --warmup 2 \
          --no-cpu-baseline --c4-steps 0 > $log 2>&1 || { echo "$label [$args] failed"; tail -5 $log; exit 1; }
      echo "$label [$args] $(tail -1 $log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    done
  done
done
