#!/bin/bash
# GPU box (r06): the auto shadow launch reads the scene's previous frame (merged for whole frames with >= 0.15
# traced shadow rays per extension ray): the full-scale tests and the shadow-launch parity tests, then the A/B
# against the build before (lib/variants/base), alternating, 3 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullscale.py "tests/test_gpu_parity.py::test_shadow_launch_modes_identical" \
    -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06_autoshadow_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06_autoshadow_pytest.log | tail -8
cp gpurun_out/parity_report.json gpurun_out/r06_autoshadow_parity.json 2>/dev/null
[ $rc -ne 0 ] && exit $rc
BASE="RT_MI355X_LIB=$PWD/buas-pathtracer_amd/lib/variants/base/librt_mi355x.so"
ARGSETS="--config c3;--config c4;--config c2" REPS=3 bash tools/gpu_ab_envs.sh "" "$BASE"
