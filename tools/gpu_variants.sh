#!/bin/bash
# GPU box: parity subset on every variant under lib/variants (PARITY_TESTS, default the parity and
# scene suites), then tools/gpu_ab.sh over the bench argument sets given.  A crash, fault or
# timeout ends the script; test failures are reported and end it too (a wrong variant is not timed).
#   PARITY_TESTS="tests/test_gpu_parity.py" REPS=2 tools/gpu_variants.sh "--config c3" "--config c4"
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for lib in buas-pathtracer_amd/lib/variants/*/librt_mi355x.so; do
  [ -f "$lib" ] || continue
  [ -n "$NO_PARITY" ] && break
  name=$(basename $(dirname $lib))
  RT_MI355X_LIB=$PWD/$lib timeout -k 10 ${PARITY_TIMEOUT:-400} python -u -m pytest ${PARITY_TESTS:-tests/test_gpu_parity.py tests/test_gpu_scenes.py} \
      -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/parity_$name.log 2>&1
  rc=$?; echo "parity $name rc=$rc: $(tail -1 gpurun_out/parity_$name.log)"
  [ $rc -ne 0 ] && { grep -E "FAILED|Error|error" gpurun_out/parity_$name.log | head -5; exit $rc; }
done
[ $# -gt 0 ] && exec_ab=1
[ -n "$exec_ab" ] && tools/gpu_ab.sh "$@"
