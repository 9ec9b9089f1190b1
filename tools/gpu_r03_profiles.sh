#!/bin/bash
# GPU box, round 3: rocprof evidence for C3 (the bench), C4 (the north star's scene) and C5 (BASELINE's roofline
# run): a rocprofv3 --kernel-trace --stats run of bench.py (kernel stats, the kernels-in-flight timeline), then every
# PMC counter group (tools/gpu_pmc_full.sh, one --pmc pass each, never combined with tracing) summarised on the box
# by tools/pmc_summary.py into $OUT/<cfg>_pmc.md and merged into $OUT/traffic.json.  Raw counter CSVs are deleted
# after the summary and the traces gzipped, so gpurun_out stays under the 64 MiB copy-back limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_TAG:-prof_r03}
mkdir -p $OUT
[ -f $OUT/traffic.json ] || cp profiles/traffic.json $OUT/traffic.json   # a later call adds its configs
for c in ${CONFIGS:-c3 c4 c5}; do
  case $c in
    c3) kt="--steps 3 --warmup 1"; pm="--steps 1 --warmup 0" ;;
    c5) kt="--config c5 --steps 1 --warmup 1"; pm="--config c5 --steps 1 --warmup 0" ;;
    *)  kt="--config $c --steps 3 --warmup 1"; pm="--config $c --steps 1 --warmup 0" ;;
  esac
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$OUT/kt_$c -o run -- \
      python3 bench.py $kt --no-cpu-baseline --c4-steps 0 > $OUT/kt_$c.log 2>&1 || { echo "trace $c failed"; tail -5 $OUT/kt_$c.log; exit 1; }
  tr=$(find $OUT/kt_$c -name "*kernel_trace.csv" | head -1); st=$(find $OUT/kt_$c -name "*kernel_stats.csv" | head -1)
  cp "$st" $OUT/${c}_kernel_stats.csv
  python3 tools/timeline.py "$tr" > $OUT/${c}_timeline.txt 2>&1
  gzip -c "$tr" > $OUT/${c}_kernel_trace.csv.gz; rm -rf $OUT/kt_$c
  echo "trace $c: $(grep -E '^frame' $OUT/${c}_timeline.txt)"
  TAG=${PROF_TAG:-prof_r03}/pmc_$c PMC_BENCH="$pm --no-cpu-baseline --c4-steps 0" tools/gpu_pmc_full.sh || { echo "pmc $c failed"; exit 1; }
  python3 tools/pmc_summary.py $OUT/pmc_$c --out $OUT/${c}_pmc.md --traffic $OUT/traffic.json --config $c \
      --bench-log $OUT/pmc_$c/pass1.log > /dev/null
  cp $OUT/pmc_$c/pass1.log $OUT/${c}_pmc_bench.log
  rm -rf $OUT/pmc_$c/pass*/
  echo "pmc $c: summarised"
done
rm -rf gpurun_out/assets
echo "profiles done"
