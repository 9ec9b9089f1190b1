#!/bin/bash
# GPU box, round 3: traversal step statistics (RT_STEP_STATS build in lib/variants/stats) for C3 and C4, and
# rocprofv3 kernel traces + stats of the bench frames of C3, C4 (north star's scene) and C5 (4K, 1024 spp),
# under gpurun_out/ev_$TAG/.  Each GPU step has its own time limit; the first failure ends the script.
#   TAG=r03 bash tools/gpu_r03_evidence.sh     (PMC: TAG=pmc_r03_c4 PMC_BENCH="--config c4 ..." tools/gpu_pmc_full.sh)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
OUT=gpurun_out/ev_$TAG
mkdir -p $OUT
STATS_LIB=$PWD/buas-pathtracer_amd/lib/variants/stats/librt_mi355x.so
for c in c3 c4; do
  RT_PARTITIONS=1 RT_DEBUG_TRAVERSAL=1 RT_MI355X_LIB=$STATS_LIB timeout -k 10 300 python bench.py --config $c \
      --spp 16 --steps 1 --warmup 0 --no-cpu-baseline --c4-steps 0 > $OUT/stats_$c.log 2>&1 || { echo "stats $c failed"; exit 1; }
  echo "stats $c:"; grep '\[rt\]' $OUT/stats_$c.log | tail -4
done
for spec in "c3:--steps 5 --warmup 1" "c4:--config c4 --steps 5 --warmup 1" "c5:--config c5 --steps 1 --warmup 1"; do
  c=${spec%%:*}; args=${spec#*:}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$OUT/prof_$c -o run -- \
      python3 bench.py $args --no-cpu-baseline --c4-steps 0 > $OUT/prof_$c.log 2>&1 || { echo "rocprof $c failed"; exit 1; }
  echo "rocprof $c: $(tail -1 $OUT/prof_$c.log | cut -c1-200)"
done
echo "evidence done"
