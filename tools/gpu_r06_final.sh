#!/bin/bash
# GPU box (r06 final): evidence part 3 (bench lines, shares, other configurations) and the final build against
# r05 (lib/variants/r05), alternating, 4 rounds: C3, C4, rank 0's share of 8.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_r06_evidence2.sh || exit 1
R05="RT_MI355X_LIB=$PWD/buas-pathtracer_amd/lib/variants/r05/librt_mi355x.so"
ARGSETS="--config c3;--config c4;--shard-of 8" REPS=4 bash tools/gpu_ab_envs.sh "" "$R05"
