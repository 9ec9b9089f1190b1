#!/bin/bash
# GPU box (r06): the fused-drain cadence test against the build without the fix (lib/variants/nofix:
# the drain_every knob only; expected to fail as r05's every-4th carry did), then the fixed default
# build with the cadence test, the integrator-switch matrix and the random scenes.
# A test failure (exit 1) continues; anything else (a fault, abort, time limit) stops the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
RT_MI355X_LIB=$PWD/buas-pathtracer_amd/lib/variants/nofix/librt_mi355x.so timeout -k 10 300 \
    python -u -m pytest tests/test_gpu_parity.py -k any_cadence -v --timeout 240 --timeout-method thread \
    > gpurun_out/r06_nofix_cadence.log 2>&1
rc=$?; echo "nofix cadence rc=$rc"; tail -5 gpurun_out/r06_nofix_cadence.log
ok $rc || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_integrator_switches.py \
    tests/test_gpu_scenes.py -k "any_cadence or switches or random_scene or fused_drain" -v --timeout 240 \
    --timeout-method thread > gpurun_out/r06_fixed.log 2>&1
rc=$?; echo "fixed rc=$rc"; tail -15 gpurun_out/r06_fixed.log
exit $rc
