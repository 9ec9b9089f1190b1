#!/bin/bash
# GPU box (r06): the merged trace launch, a third of its blocks on the shadow queue after (or before,
# RT_SHADOW_FIRST=1) their extension items, against the separate connect launch (lib/variants/sep).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SEP="RT_MI355X_LIB=$PWD/buas-pathtracer_amd/lib/variants/sep/librt_mi355x.so"
RT_SHADOW_PCT=33 RT_SHADOW_FIRST=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused_drain or frame_bitwise" \
    -x -q --timeout 240 --timeout-method thread > gpurun_out/r06_shpct2_tests.log 2>&1 || { tail -5 gpurun_out/r06_shpct2_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r06_shpct2_tests.log
ARGSETS="--config c3;--config c4;--shard-of 8" REPS=3 bash tools/gpu_ab_envs.sh "RT_SHADOW_PCT=33" "RT_SHADOW_PCT=33 RT_SHADOW_FIRST=1" "$SEP"
