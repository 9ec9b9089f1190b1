#!/bin/bash
# GPU box: the -m gpu suite of the working tree's build (log under gpurun_out/${TAG}_pytest.log),
# then, unless it crashed, tools/gpu_ab.sh over the argument sets given (REPS alternating rounds).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
tag=${TAG:-t}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 170 \
    --timeout-method thread ${PYTEST_ARGS} > gpurun_out/${tag}_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/${tag}_pytest.log | tail -12
cp gpurun_out/parity_report.json gpurun_out/${tag}_parity_report.json 2>/dev/null
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
[ $# -gt 0 ] && REPS=${REPS:-2} tools/gpu_ab.sh "$@"
