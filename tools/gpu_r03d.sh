#!/bin/bash
# GPU box: tools/gpu_r03b.sh (tests + A/B against lib/variants/*), then tools/gpu_sweep_args.sh with the arguments.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_r03b.sh || exit $?
[ $# -gt 0 ] || exit 0
REPS=${SWEEP_REPS:-2} tools/gpu_sweep_args.sh "$@"
