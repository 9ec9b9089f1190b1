#!/bin/bash
# GPU box (r06): a missing path's environment texel fetched into LDS at k_shade's start (global_load_lds_dwordx3):
# parity, edge (+ the plane-batch rooms) and scene tests, then the A/B against the build before
# (lib/variants/base), alternating, 3 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_scenes.py \
    -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/r06_skypre_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06_skypre_pytest.log | tail -8
[ $rc -ne 0 ] && exit $rc
BASE="RT_MI355X_LIB=$PWD/buas-pathtracer_amd/lib/variants/base/librt_mi355x.so"
ARGSETS="--config c3;--config c4;--shard-of 8" REPS=3 bash tools/gpu_ab_envs.sh "" "$BASE"
