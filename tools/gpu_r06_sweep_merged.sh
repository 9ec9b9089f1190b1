#!/bin/bash
# GPU box (r06 final build): the merged launch's knobs on the whole C3 frame (merged from its second frame): the
# share of trace blocks taking shadow items (RT_SHADOW_PCT, 33) and the trace grid (RT_TRACE_GRID_PCT, 75), 2 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGSETS="--config c3;--shard-of 8" REPS=2 bash tools/gpu_ab_envs.sh "" "RT_SHADOW_PCT=25" "RT_SHADOW_PCT=50" \
    "RT_TRACE_GRID_PCT=87" "RT_TRACE_GRID_PCT=62"
