#!/bin/bash
# Full bench (C3, 1080p 256spp) + rocprofv3 kernel-trace stats of a shorter run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOTDIR=$(pwd)
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 ${BENCH_TIMEOUT:-700} python bench.py ${BENCH_ARGS:---steps 3 --warmup 1} > gpurun_out/bench_${TAG}.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_${TAG}.log
[ $rc -ne 0 ] && exit $rc
if [ -n "$PROF_ARGS" ]; then
  export TMPDIR=/tmp
  timeout -k 10 ${PROF_TIMEOUT:-500} rocprofv3 --kernel-trace --stats --output-format csv -d $ROOTDIR/gpurun_out/prof_${TAG} -o run -- python3 $ROOTDIR/bench.py $PROF_ARGS > gpurun_out/prof_${TAG}.log 2>&1
  prc=$?; echo "rocprof rc=$prc"; tail -3 gpurun_out/prof_${TAG}.log
  find gpurun_out/prof_${TAG} -name "*stats*" | head
  exit $prc
fi
