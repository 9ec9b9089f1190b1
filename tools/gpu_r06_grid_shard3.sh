#!/bin/bash
# GPU box (r06): a rank's share of 8 with the small-pool trace grid at 37 / 31 / 25 % of a wave (RT_TRACE_GRID_PCT
# 56 / 47 / 38, two thirds taken) against the default 50 %, 3 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGSETS="--shard-of 8" REPS=3 bash tools/gpu_ab_envs.sh "" "RT_TRACE_GRID_PCT=56" "RT_TRACE_GRID_PCT=47" "RT_TRACE_GRID_PCT=38"
