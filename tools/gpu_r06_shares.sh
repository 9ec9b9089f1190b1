#!/bin/bash
# GPU box (r06): per-rank cost of the two shard modes (bench.py --shard-of 8): sample passes (bench.py's
# default) and the north star's tiles t % 8, ranks 0 and 7, alternating, 2 rounds; the host's rounds
# (RT_DEBUG_TIMING) of one pass share.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/shares
for rep in 1 2; do
  for mode in passes tiles; do
    for r in 0 7; do
      log=gpurun_out/shares/${mode}_${r}_$rep.log
      timeout -k 10 200 python bench.py --shard-of 8 --shard-index $r --shard-mode $mode --steps 5 --warmup 2 \
          --no-cpu-baseline --c4-steps 0 > $log 2>&1 || { echo "$mode $r failed"; tail -3 $log; exit 1; }
      echo "$mode rank $r: $(tail -1 $log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "Mrays/s", d["ms_per_step"], "ms", d["samples_per_s"], "samples/s")')"
    done
  done
done
RT_DEBUG_TIMING=1 timeout -k 10 200 python bench.py --shard-of 8 --steps 2 --warmup 1 --no-cpu-baseline --c4-steps 0 \
    > gpurun_out/shares/host_rounds.log 2>&1 || exit 1
grep -A10 "host rounds" gpurun_out/shares/host_rounds.log | tail -11
