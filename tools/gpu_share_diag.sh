#!/bin/bash
# GPU box: where a small share's time goes.  RT_DEBUG_TIMING host timestamps of a rank-0-of-8 frame, and a
# rocprofv3 kernel trace of the same bench, summarised by tools/timeline.py in 1 ms buckets.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/share_diag
mkdir -p $OUT
ARGS=${ARGS:-"--config c3 --shard-of 8"}
RT_DEBUG_TIMING=1 timeout -k 10 300 python bench.py $ARGS --steps 3 --warmup 1 --no-cpu-baseline --c4-steps 0 \
    > $OUT/timing.log 2>&1 || { echo "timing run failed"; tail -5 $OUT/timing.log; exit 1; }
grep "rt timing" $OUT/timing.log | tail -12; tail -1 $OUT/timing.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $PWD/$OUT/kt -o run -- \
    python3 bench.py $ARGS --steps 3 --warmup 1 --no-cpu-baseline --c4-steps 0 > $OUT/kt.log 2>&1 || { echo "trace failed"; exit 1; }
tr=$(find $OUT/kt -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py "$tr" --bucket-ms ${BUCKET:-1} | tee $OUT/timeline.txt
gzip -c "$tr" > $OUT/kernel_trace.csv.gz; rm -rf $OUT/kt
