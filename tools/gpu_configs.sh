#!/bin/bash
# GPU box: per-rank shard timings (bench --shard-of) and one bench line per BASELINE config.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for n in ${SHARDS:-2 4}; do
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --shard-of $n > gpurun_out/sh_$n.log 2>&1 || exit 1
  tail -1 gpurun_out/sh_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('shard-of', $n, d['value'], d['ms_per_step'])"
done
for c in ${CONFIGS:-c1 c2 c4}; do
  timeout -k 10 400 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1 || exit 1
  tail -1 gpurun_out/bench_$c.log | cut -c1-300
done
if [ -n "$C5" ]; then
  timeout -k 10 600 python bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1
  rc=$?; echo "c5 rc=$rc"; tail -1 gpurun_out/bench_c5.log | cut -c1-300; exit $rc
fi
