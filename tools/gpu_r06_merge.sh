#!/bin/bash
# GPU box (r06): the whole -m gpu suite on the working tree's library (shadow rays traced in the next
# iteration's k_trace launch), then the A/B against lib/variants/sep (the separate connect launch).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread \
    > gpurun_out/r06_merge_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06_merge_pytest.log | tail -8
cp gpurun_out/parity_report.json gpurun_out/r06_merge_parity_report.json 2>/dev/null
[ $rc -ne 0 ] && exit $rc
REPS=${REPS:-2} bash tools/gpu_ab.sh "--config c3" "--config c4" "--shard-of 8"
