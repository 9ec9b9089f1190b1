#!/bin/bash
# GPU box (r06 final build): the fused-drain threshold (live paths at which k_drain takes a partition's last paths;
# auto: max(2.5 x the drain grid's lanes, a tenth of the pool) = ~330k for a share of 8, 840k for the whole frame)
# at 250k / 500k / 1.2M, 2 rounds, rank 0's share of 8 and the whole C3 frame.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGSETS="--shard-of 8;--config c3" REPS=2 bash tools/gpu_ab_envs.sh "" "RT_FUSE_PATHS=250000" "RT_FUSE_PATHS=500000" "RT_FUSE_PATHS=1200000"
