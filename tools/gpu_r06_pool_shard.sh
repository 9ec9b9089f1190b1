#!/bin/bash
# GPU box (r06): a rank's share of 8 with path pools of 2.0M / 2.6M / 4.2M paths against the default (a fifth of the
# partition's samples: 3.3M), 3 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGSETS="--shard-of 8;--shard-of 8 --pool 2097152;--shard-of 8 --pool 2621440;--shard-of 8 --pool 4194304" REPS=3 \
    bash tools/gpu_ab_envs.sh ""
