#!/bin/bash
# GPU box (r06): rank 0's share of a C4 frame (2, 4, 8 ranks) with the separate / merged shadow launch.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGSETS="--config c4 --shard-of 8;--config c4 --shard-of 4;--config c4 --shard-of 2" REPS=2 bash tools/gpu_ab_envs.sh \
    "RT_SHADOW_LAUNCH=1" "RT_SHADOW_LAUNCH=2"
