#!/bin/bash
# GPU box (r06): pools under 4M paths take two thirds of the trace grid, against the fixed grid
# (RT_TRACE_GRID_BY_POOL=0), alternating, 4 rounds: ranks 0 and 7 of 8 (3.3M paths) and C1 (2M).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGSETS="--shard-of 8;--shard-of 8 --shard-index 7;--config c1" REPS=4 bash tools/gpu_ab_envs.sh "" "RT_TRACE_GRID_BY_POOL=0"
