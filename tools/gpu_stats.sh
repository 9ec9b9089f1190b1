#!/bin/bash
# GPU box: traversal step statistics (RT_STEP_STATS build in lib/variants/stats), one partition, 16 spp.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
RT_PARTITIONS=1 RT_DEBUG_TRAVERSAL=1 RT_MI355X_LIB=$PWD/buas-pathtracer_amd/lib/variants/stats/librt_mi355x.so timeout -k 10 300 python bench.py --spp 16 --steps 1 --warmup 0 --no-cpu-baseline ${STATS_ARGS} > gpurun_out/stats.log 2>&1 || exit 1
grep '\[rt\]' gpurun_out/stats.log | tail -4
