#!/bin/bash
# GPU box (r06): where a rank's share of 8 loses time (kernel + memory-copy trace, the host's rounds),
# then the drain-carry cadence A/B (RT_DRAIN_EVERY) on C3, C4 and the share of 8.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
RT_DEBUG_TIMING=1 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
    -d $PWD/gpurun_out/r06_s8trace -o run -- python3 bench.py --shard-of 8 --steps 2 --warmup 1 \
    --no-cpu-baseline --c4-steps 0 > gpurun_out/r06_s8trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r06_s8trace.log; exit $rc; }
f=$(find gpurun_out/r06_s8trace -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py "$f" --bucket-ms 1 > gpurun_out/r06_s8_timeline.txt 2>&1
cat gpurun_out/r06_s8_timeline.txt
grep -A12 "host rounds" gpurun_out/r06_s8trace.log | tail -12
bash tools/gpu_ab_envs.sh "" "RT_DRAIN_EVERY=2" "RT_DRAIN_EVERY=3"
