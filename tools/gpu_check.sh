#!/bin/bash
# GPU box: smoke -> the -m gpu suite -> a short C3 bench.  Test failures (pytest rc 1) do not stop
# the sequence; a crash, a fault or a timeout does.
#   TAG=r02b PYTEST_ARGS="tests/test_gpu_parity.py" BENCH_ARGS="--steps 5 --warmup 2" tools/gpu_check.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-check}
mkdir -p gpurun_out
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_${TAG}.log
[ $rc -ne 0 ] && exit $rc
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest ${PYTEST_ARGS:-tests} -m gpu -v -p no:cacheprovider \
      --timeout 300 --timeout-method thread --maxfail=${MAXFAIL:-20} > gpurun_out/pytest_gpu_${TAG}.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_gpu_${TAG}.log | tail -3
  cp gpurun_out/parity_report.json gpurun_out/parity_report_${TAG}.json 2>/dev/null
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ -n "$BENCH_ARGS" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py $BENCH_ARGS > gpurun_out/bench_${TAG}.log 2>&1
  brc=$?; echo "bench rc=$brc"; tail -1 gpurun_out/bench_${TAG}.log | cut -c1-700
  exit $brc
fi
exit $rc
