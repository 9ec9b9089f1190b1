#!/bin/bash
# GPU box (r06): with the record ring sized by the path life, the merged trace launch (a third of the blocks
# on the shadow queue after their extension items; all blocks, shadow items first) against the separate
# connect launch (lib/variants/sep, the same ring), on C3, C4 and rank 0's share of 8.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SEP="RT_MI355X_LIB=$PWD/buas-pathtracer_amd/lib/variants/sep/librt_mi355x.so"
ARGSETS="--config c4;--config c3;--shard-of 8" REPS=2 bash tools/gpu_ab_envs.sh "RT_SHADOW_PCT=33" "RT_SHADOW_FIRST=1" "$SEP"
