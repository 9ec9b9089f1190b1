#!/bin/bash
# GPU box: parity tests, then the variant sweep (tools/gpu_variants.sh). Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E 'FAILED|ERROR|passed|failed' gpurun_out/pytest_gpu.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ -n "$NO_VARIANTS" ] && exit $rc
bash tools/gpu_variants.sh
