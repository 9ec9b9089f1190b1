#!/bin/bash
# GPU box (r06 evidence, part 1): smoke, the -m gpu suite and its parity report, the default bench line (CPU
# baseline included), rocprofv3 kernel traces + stats of C3 (no C4 frames) and C4, and a C3 timeline.
# Each GPU step has its own time limit; the first failure that is not a test failure ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r06}
OUT=gpurun_out/ev_$TAG
mkdir -p $OUT
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" $OUT/pytest_gpu.log | tail -5
cp gpurun_out/parity_report.json $OUT/parity_report.json 2>/dev/null
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-240
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$OUT/prof_c3 -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --c4-steps 0 > $OUT/prof_c3.log 2>&1 || { echo "rocprof c3 failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$OUT/prof_c4 -o run -- \
    python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof_c4.log 2>&1 || { echo "rocprof c4 failed"; exit 1; }
f=$(find $OUT/prof_c3 -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py "$f" --bucket-ms 5 > $OUT/c3_timeline.txt 2>&1
echo "evidence part 1 done"
