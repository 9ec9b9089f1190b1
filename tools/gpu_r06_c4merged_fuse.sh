#!/bin/bash
# GPU box (r06): C4 with the merged shadow launch and an earlier fused drain (RT_FUSE_PATHS 1.2M / 2M; auto 840k)
# against the auto choice (separate), 2 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGSETS="--config c4" REPS=2 bash tools/gpu_ab_envs.sh "" "RT_SHADOW_LAUNCH=2" "RT_SHADOW_LAUNCH=2 RT_FUSE_PATHS=1200000" \
    "RT_SHADOW_LAUNCH=2 RT_FUSE_PATHS=2000000" "RT_SHADOW_LAUNCH=2 RT_FUSE_PATHS=500000"
