#!/bin/bash
# GPU box: the default build against every variant under lib/variants, alternating REPS times (default 2),
# for each bench.py argument set given as one quoted string, e.g.
#   tools/gpu_ab.sh "--config c3" "--config c3 --shard-of 8"
# Prints one line per run: variant, argument set, Mrays/s, ms per frame.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
for rep in $(seq 1 ${REPS:-2}); do
  k=0
  for args in "$@"; do
    k=$((k + 1))
    for lib in buas-pathtracer_amd/lib/librt_mi355x.so buas-pathtracer_amd/lib/variants/*/librt_mi355x.so; do
      [ -f "$lib" ] || continue
      name=$(basename $(dirname $lib)); [ "$name" = lib ] && name=default
      log=gpurun_out/ab/${name}_${k}_${rep}.log
      RT_MI355X_LIB=$PWD/$lib timeout -k 10 300 python bench.py $args --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline \
          --c4-steps 0 > $log 2>&1 || { echo "$name [$args] failed"; tail -5 $log; exit 1; }
      echo "$name [$args] $(tail -1 $log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    done
  done
done
