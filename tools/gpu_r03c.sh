#!/bin/bash
# GPU box: tools/gpu_r03b.sh (tests + A/B against lib/variants/*), then the bench once per environment setting
# given as arguments (tools/gpu_ab_env.sh, no tests).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_r03b.sh || exit $?
[ $# -gt 0 ] || exit 0
NO_TESTS=1 BENCH_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --c4-steps 0" bash tools/gpu_ab_env.sh "$@"
