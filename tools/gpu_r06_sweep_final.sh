#!/bin/bash
# GPU box (r06 final build): the launch settings again after the batched prologue: the merged shadow launch for
# whole frames, the trace grid (75 % of a full-occupancy wave by default) and the separate shadow launch's grid
# (25 %), alternating, 2 rounds, C3 and C4.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGSETS="--config c3;--config c4" REPS=2 bash tools/gpu_ab_envs.sh "" "RT_SHADOW_LAUNCH=2" "RT_TRACE_GRID_PCT=100" \
    "RT_CONNECT_GRID_PCT=33" "RT_PARTITIONS=5"
