#!/bin/bash
# GPU box: the evidence set of a build, under gpurun_out/ev_$TAG/ (copied into profiles/ afterwards):
#   the -m gpu suite and its parity report, the default bench line (with the CPU baseline), a rocprofv3
#   kernel trace + stats of the bench, and the other configurations and per-rank shares.
# Each GPU step has its own time limit; the first failure that is not a test failure ends the script.
#   TAG=r02f bash tools/gpu_evidence.sh      (then TAG=pmc_r02f bash tools/gpu_pmc_full.sh in its own call)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-ev}
OUT=gpurun_out/ev_$TAG
mkdir -p $OUT
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $OUT/pytest_gpu.log | tail -1
cp gpurun_out/parity_report.json $OUT/parity_report.json 2>/dev/null
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; exit 1; }
tail -1 $OUT/bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$OUT/prof -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
for n in 2 4 8; do
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --shard-of $n > $OUT/shard_$n.log 2>&1 || exit 1
  echo "shard-of $n: $(tail -1 $OUT/shard_$n.log | cut -c1-160)"
done
for c in c1 c2 c4 c4i; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_$c.log 2>&1 || exit 1
done
timeout -k 10 400 python bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench_c5.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --env-sampling 1 > $OUT/bench_c3_env.log 2>&1 || exit 1
echo "evidence done"
