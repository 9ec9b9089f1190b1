#!/bin/bash
# GPU box (r06): the r06 build without k_generate's done check against r05 (lib/variants/r05), and with r05's
# record ring (RT_SPLAT_RING=39), alternating, 3 rounds: C3, C4.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R05="RT_MI355X_LIB=$PWD/buas-pathtracer_amd/lib/variants/r05/librt_mi355x.so"
ARGSETS="--config c3;--config c4" REPS=3 bash tools/gpu_ab_envs.sh "" "$R05" "RT_SPLAT_RING=39"
