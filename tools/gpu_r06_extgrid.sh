#!/bin/bash
# GPU box (r06): the separate schedule's extension launch on 83 % of the trace grid (62 % of a wave) against the
# full grid (RT_TRACE_GRID_EXT_PCT=100), 4 rounds: C4, C4i, and C3 forced separate (RT_SHADOW_LAUNCH=1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGSETS="--config c4;--config c4i" REPS=4 bash tools/gpu_ab_envs.sh "" "RT_TRACE_GRID_EXT_PCT=100" && \
ARGSETS="--config c3" REPS=3 bash tools/gpu_ab_envs.sh "RT_SHADOW_LAUNCH=1" "RT_SHADOW_LAUNCH=1 RT_TRACE_GRID_EXT_PCT=100"
