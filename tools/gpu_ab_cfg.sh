#!/bin/bash
# GPU box: the default build against every variant under lib/variants, alternating twice, on the bench
# configurations given (bench.py --config), e.g. tools/gpu_ab_cfg.sh c4 c4i c2
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/variants
for rep in 1 2; do
  for cfg in "$@"; do
    for lib in buas-pathtracer_amd/lib/librt_mi355x.so buas-pathtracer_amd/lib/variants/*/librt_mi355x.so; do
      [ -f "$lib" ] || continue
      name=$(basename $(dirname $lib)); [ "$name" = lib ] && name=default
      RT_MI355X_LIB=$PWD/$lib timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline \
          > gpurun_out/variants/${name}_$cfg.log 2>&1 || { echo "$name $cfg failed"; exit 1; }
      echo "$name $cfg $(tail -1 gpurun_out/variants/${name}_$cfg.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["traced_rays"])')"
    done
  done
done
