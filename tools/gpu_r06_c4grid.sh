#!/bin/bash
# GPU box (r06 final build): C4's launch grids (separate shadow launch): the trace grid at 62 % of a wave
# (RT_TRACE_GRID_PCT, 75) and the shadow launch's at 20 / 15 % (RT_CONNECT_GRID_PCT, 25), 3 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGSETS="--config c4" REPS=3 bash tools/gpu_ab_envs.sh "" "RT_TRACE_GRID_PCT=62" "RT_CONNECT_GRID_PCT=20" "RT_CONNECT_GRID_PCT=15"
