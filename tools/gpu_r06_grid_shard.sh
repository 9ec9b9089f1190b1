#!/bin/bash
# GPU box (r06 final build): the trace grid for a rank's share (RT_TRACE_GRID_PCT, 75 % of a full-occupancy wave of
# blocks by default) at 62 % and 50 %, shares of 8 and 4, 3 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGSETS="--shard-of 8;--shard-of 4" REPS=3 bash tools/gpu_ab_envs.sh "" "RT_TRACE_GRID_PCT=62" "RT_TRACE_GRID_PCT=50"
