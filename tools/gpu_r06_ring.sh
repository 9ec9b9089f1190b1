#!/bin/bash
# GPU box (r06): does the record ring throttle the claims of the merged trace launch (records written
# an iteration later)?  C4 / C3 with a larger ring (RT_SPLAT_RING=60) against the default, merged
# (RT_SHADOW_PCT=33) and separate (lib/variants/sep).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SEP="RT_MI355X_LIB=$PWD/buas-pathtracer_amd/lib/variants/sep/librt_mi355x.so"
ARGSETS="--config c4;--config c3" REPS=2 bash tools/gpu_ab_envs.sh "RT_SHADOW_PCT=33" "RT_SHADOW_PCT=33 RT_SPLAT_RING=60" \
    "$SEP" "$SEP RT_SPLAT_RING=60"
