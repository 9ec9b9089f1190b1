#!/bin/bash
# GPU box, round 3 (session 2): the -m gpu suite on the working build, then an A/B of the working build
# against lib/variants/* (tools/gpu_ab.sh).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-r03b}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
      > gpurun_out/pytest_gpu_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_$TAG.log
  cp gpurun_out/parity_report.json gpurun_out/parity_report_$TAG.json 2>/dev/null
  [ $rc -ne 0 ] && exit $rc
fi
REPS=${REPS:-2} tools/gpu_ab.sh "--config c3" "--config c3 --shard-of 8" "--config c4"
