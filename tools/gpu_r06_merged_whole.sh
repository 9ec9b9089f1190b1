#!/bin/bash
# GPU box (r06 final build): the merged shadow launch on whole frames (RT_SHADOW_LAUNCH=2) against the auto policy
# (separate for whole frames), 4 rounds, C3 and C2 (Cornell box scenes) and C4.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGSETS="--config c3;--config c2;--config c4" REPS=4 bash tools/gpu_ab_envs.sh "" "RT_SHADOW_LAUNCH=2"
