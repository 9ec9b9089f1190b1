#!/bin/bash
# GPU box: the default build and every variant under lib/variants, alternating twice, on the full C3 frame
# and rank 0's share of 4- and 8-rank frames (--shard-of).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/variants
for rep in 1 2; do
  for lib in buas-pathtracer_amd/lib/librt_mi355x.so buas-pathtracer_amd/lib/variants/*/librt_mi355x.so; do
    [ -f "$lib" ] || continue
    name=$(basename $(dirname $lib)); [ "$name" = lib ] && name=default
    for mode in full s4 s8; do
      extra=""; [ $mode = s4 ] && extra="--shard-of 4"; [ $mode = s8 ] && extra="--shard-of 8"
      RT_MI355X_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline $extra \
          > gpurun_out/variants/${name}_$mode.log 2>&1 || { echo "$name $mode failed"; exit 1; }
      echo "$name $mode $(tail -1 gpurun_out/variants/${name}_$mode.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    done
  done
done
