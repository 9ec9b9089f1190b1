#!/bin/bash
# GPU box (r06): shares of 2 and 4 on the final build against the batched-prologue build (lib/variants/base), 3 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
BASE="RT_MI355X_LIB=$PWD/buas-pathtracer_amd/lib/variants/base/librt_mi355x.so"
ARGSETS="--shard-of 2;--shard-of 4" REPS=3 bash tools/gpu_ab_envs.sh "" "$BASE"
