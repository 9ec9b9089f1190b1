#!/bin/bash
# GPU box: rocprofv3 kernel traces of the full C3 frame and of rank 0's share of 2/8-rank frames,
# for tools/drain.py (per-partition iteration timelines).  TAG=x bash tools/gpu_drain.sh [tests]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-drain}
OUT=gpurun_out/drain_$TAG
mkdir -p $OUT
if [ "$1" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread \
      > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  grep -E "passed|failed" $OUT/pytest_gpu.log | tail -1
fi
for n in 8 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $PWD/$OUT/prof_s$n -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --shard-of $n > $OUT/bench_s$n.log 2>&1 \
      || { echo "rocprof shard $n failed"; tail -20 $OUT/bench_s$n.log; exit 1; }
  echo "shard-of $n: $(tail -1 $OUT/bench_s$n.log | cut -c1-200)"
done
echo done
