#!/bin/bash
# GPU box (r06): k_shade wave time per section (tools/shade_sections.patch built as lib/variants/shadeprof),
# C3 and C4 1080p 256 spp, one warm-up and two timed frames each (the probe prints one line per frame).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for c in c3 c4; do
  RT_MI355X_LIB=$PWD/buas-pathtracer_amd/lib/variants/shadeprof/librt_mi355x.so timeout -k 10 300 \
      python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --c4-steps 0 > gpurun_out/r06_shadeprof_$c.log 2>&1 \
      || { echo "$c failed"; tail -5 gpurun_out/r06_shadeprof_$c.log; exit 1; }
  echo "== $c"; grep shade_prof gpurun_out/r06_shadeprof_$c.log
  tail -1 gpurun_out/r06_shadeprof_$c.log | cut -c1-200
done
