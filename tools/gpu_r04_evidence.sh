#!/bin/bash
# GPU box: the r04 evidence set of the working tree's build, under gpurun_out/ev_$TAG/ (copied into
# profiles/ afterwards): smoke, the -m gpu suite and its parity report, the default bench line (CPU
# baseline included), a rocprofv3 kernel trace + stats of the C3 and C4 benches, the pass shares of
# 2 / 4 / 8 ranks (rank 0 and rank 7 of 8) with a kernel trace of rank 0 of 8, and the other configs.
# Every GPU step has its own time limit; the first failure that is not a test failure ends the script.
#   TAG=r04 tools/gpu_r04_evidence.sh          (PMC: TAG=pmc_r04_c3 PMC_BENCH=... tools/gpu_pmc_full.sh)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
OUT=gpurun_out/ev_$TAG
mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step smoke
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
if [ -z "$SKIP_TESTS" ]; then
  step pytest
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 170 --timeout-method thread \
      > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $OUT/pytest_gpu.log | tail -1
  cp gpurun_out/parity_report.json $OUT/parity_report.json 2>/dev/null
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
step bench
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-400
for c in c3 c4; do
  step "rocprof $c"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$OUT/prof_$c -o run -- \
      python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --c4-steps 0 > $OUT/prof_$c.log 2>&1 \
      || { echo "rocprof $c failed"; tail -5 $OUT/prof_$c.log; exit 1; }
done
for n in 2 4 8; do
  step "share of $n"
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --c4-steps 0 --shard-of $n > $OUT/shard_$n.log 2>&1 || exit 1
  echo "shard-of $n: $(tail -1 $OUT/shard_$n.log | cut -c1-200)"
done
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --c4-steps 0 --shard-of 8 --shard-index 7 > $OUT/shard_8_r7.log 2>&1 || exit 1
step "rocprof share of 8"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $PWD/$OUT/prof_shard8 -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --c4-steps 0 --shard-of 8 > $OUT/prof_shard8.log 2>&1 || exit 1
for c in c1 c2 c4i c5; do
  step "config $c"
  s=3; [ $c = c5 ] && s=1
  timeout -k 10 300 python bench.py --config $c --steps $s --warmup 1 --no-cpu-baseline --c4-steps 0 > $OUT/bench_$c.log 2>&1 || exit 1
done
step done
