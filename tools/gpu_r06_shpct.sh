#!/bin/bash
# GPU box (r06): the merged trace launch with all / half / a third of its blocks taking the shadow queue
# (RT_SHADOW_PCT), against the separate connect launch (lib/variants/sep).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SEP="RT_MI355X_LIB=$PWD/buas-pathtracer_amd/lib/variants/sep/librt_mi355x.so"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused_drain or stream_splat_deterministic or frame_bitwise" \
    -x -q --timeout 240 --timeout-method thread > gpurun_out/r06_shpct_tests.log 2>&1 || { tail -5 gpurun_out/r06_shpct_tests.log; exit 1; }
RT_SHADOW_PCT=33 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused_drain or frame_bitwise" \
    -x -q --timeout 240 --timeout-method thread >> gpurun_out/r06_shpct_tests.log 2>&1 || { tail -5 gpurun_out/r06_shpct_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r06_shpct_tests.log
bash tools/gpu_ab_envs.sh "" "RT_SHADOW_PCT=50" "RT_SHADOW_PCT=33" "$SEP"
