#!/bin/bash
# GPU box (r06): k_shade at 8 waves per SIMD (64 VGPRs, 78 SGPRs: 17 SGPRs spilled to VGPR lanes) against 7
# (lib/variants/w7: 72 VGPRs, no spills), alternating, 3 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
W7="RT_MI355X_LIB=$PWD/buas-pathtracer_amd/lib/variants/w7/librt_mi355x.so"
ARGSETS="--config c3;--config c4;--shard-of 8" REPS=3 bash tools/gpu_ab_envs.sh "" "$W7"
