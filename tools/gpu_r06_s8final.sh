#!/bin/bash
# GPU box (r06 final build): rank 0's share of 8 under rocprofv3 --kernel-trace (kernel stats and a 1 ms timeline of
# the second frame): the merged launch and the small-pool trace grid.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/r06_s8final -o run -- \
    python3 bench.py --shard-of 8 --steps 2 --warmup 1 --no-cpu-baseline --c4-steps 0 > gpurun_out/r06_s8final.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r06_s8final.log; exit $rc; }
f=$(find gpurun_out/r06_s8final -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py "$f" --bucket-ms 1 > gpurun_out/r06_s8final_timeline.txt 2>&1
head -20 gpurun_out/r06_s8final_timeline.txt
