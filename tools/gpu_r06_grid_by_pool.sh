#!/bin/bash
# GPU box (r06): the trace grid scaled by sqrt(pool / 4 x 2^21) against the fixed grid (RT_TRACE_GRID_BY_POOL=0),
# alternating, 3 rounds: shares of 8 and 4, the whole C3 frame (unchanged: the largest pool) and C1 (a small frame).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGSETS="--shard-of 8;--shard-of 4;--config c3;--config c1" REPS=3 bash tools/gpu_ab_envs.sh "" "RT_TRACE_GRID_BY_POOL=0"
