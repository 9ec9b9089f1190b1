#!/bin/bash
# r04 GPU session: the GPU suite, then an A/B of the working tree's library against every variant
# under lib/variants (REPS alternating pairs), C3 and C4.  Stops at a crash, abort or time limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
tag=${TAG:-r04a}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 170 \
      --timeout-method thread ${PYTEST_ARGS} > gpurun_out/${tag}_pytest.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -30 gpurun_out/${tag}_pytest.log
  cp gpurun_out/parity_report.json gpurun_out/${tag}_parity_report.json 2>/dev/null
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
fi
if [ -n "$AB" ]; then                  # AB=1: C3 and C4 frames
  REPS=${REPS:-2} tools/gpu_ab.sh "--config c3" "--config c4" || exit 1
fi
