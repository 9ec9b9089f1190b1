#!/bin/bash
# GPU box (r06): the record ring on the whole C3 / C4 frames: r05's ring (C3: 16 + 21 + 2 = 39 passes), 48, and the
# r06 default (the path-life formula: 64 = the partition's passes for both), against r05 (lib/variants/r05), 3 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R05="RT_MI355X_LIB=$PWD/buas-pathtracer_amd/lib/variants/r05/librt_mi355x.so"
ARGSETS="--config c3;--config c4" REPS=3 bash tools/gpu_ab_envs.sh "" "RT_SPLAT_RING=39" "RT_SPLAT_RING=48" "$R05"
