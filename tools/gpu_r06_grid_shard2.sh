#!/bin/bash
# GPU box (r06): a rank's share of 8 with the small-pool trace grid at 37 % / 43 % of a wave (RT_TRACE_GRID_PCT 56 / 65,
# two thirds taken) against the default 50 %, and the drain grid at 75 % (RT_DRAIN_GRID_PCT), 3 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGSETS="--shard-of 8" REPS=3 bash tools/gpu_ab_envs.sh "" "RT_TRACE_GRID_PCT=56" "RT_TRACE_GRID_PCT=65" "RT_DRAIN_GRID_PCT=75"
