#!/bin/bash
# GPU box (r06): the whole -m gpu suite with rt_scene_config::shadow_launch (auto: merged for pools
# under 4M paths), then the A/B of the two forced modes against auto on C3, C4 and rank 0's shares of
# 2, 4 and 8 (RT_SHADOW_LAUNCH=1 separate, 2 merged).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread \
    > gpurun_out/r06_modes_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06_modes_pytest.log | tail -8
cp gpurun_out/parity_report.json gpurun_out/r06_modes_parity_report.json 2>/dev/null
[ $rc -ne 0 ] && exit $rc
ARGSETS="--config c3;--config c4;--shard-of 8;--shard-of 4;--shard-of 2" REPS=2 bash tools/gpu_ab_envs.sh "" "RT_SHADOW_LAUNCH=1" "RT_SHADOW_LAUNCH=2"
