#!/bin/bash
# GPU box, round 3: the -m gpu suite, then an A/B of the working build against lib/variants/head, then the evidence
# set (tools/gpu_r03_evidence.sh).  Stops at the first failure that is not a test failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-r03}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_$TAG.log
cp gpurun_out/parity_report.json gpurun_out/parity_report_$TAG.json 2>/dev/null
[ $rc -ne 0 ] && exit $rc
if [ -z "$NO_AB" ]; then
  mkdir -p gpurun_out/ab_keep; rm -rf gpurun_out/ab
  REPS=${REPS:-2} tools/gpu_ab.sh "--config c3" "--config c3 --shard-of 8" "--config c4" || exit 1
fi
[ -n "$NO_EVIDENCE" ] && exit 0
TAG=$TAG bash tools/gpu_r03_evidence.sh
