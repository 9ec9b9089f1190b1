#!/bin/bash
# GPU box (r06 evidence, part 3): the default bench line with the refreshed profiles/traffic.json, the driver's
# 20-step form, rank 0's pass shares of 2 / 4 / 8 (rank 7 of 8 too) and the tile share of 8, the other configurations.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ev_r06b
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-200
timeout -k 10 400 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $OUT/bench20.log 2>&1 || { echo "bench20 failed"; exit 1; }
tail -1 $OUT/bench20.log | cut -c1-200
for n in 2 4 8; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --c4-steps 0 --shard-of $n > $OUT/shard_$n.log 2>&1 || exit 1
  echo "pass share of $n (rank 0): $(tail -1 $OUT/shard_$n.log | cut -c1-150)"
done
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --c4-steps 0 --shard-of 8 --shard-index 7 > $OUT/shard_8_r7.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --c4-steps 0 --shard-of 8 --shard-mode tiles > $OUT/shard_8_tiles.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --c4-steps 0 --shard-of 8 --shard-mode tiles --shard-index 7 > $OUT/shard_8_tiles_r7.log 2>&1 || exit 1
for c in c1 c2 c4 c4i; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --c4-steps 0 > $OUT/bench_$c.log 2>&1 || exit 1
done
timeout -k 10 400 python bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline --c4-steps 0 > $OUT/bench_c5.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --c4-steps 0 --env-sampling 1 > $OUT/bench_c3_env.log 2>&1 || exit 1
echo "evidence part 3 done"
