#!/bin/bash
# GPU box (r06 evidence, part 2): the PMC passes of one C3 frame and one C4 frame (tools/gpu_pmc_full.sh), for
# profiles/traffic.json (tools/pmc_summary.py --traffic) and the per-kernel summaries.  C3 with the merged shadow
# launch: the bench's timed C3 frames run it (the auto policy, from a scene's second frame), while a one-frame pass
# would be the scene's first frame (separate).  C4 runs separate either way.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
RT_SHADOW_LAUNCH=2 TAG=pmc_r06_c3 PMC_BENCH="--steps 1 --warmup 0 --no-cpu-baseline" bash tools/gpu_pmc_full.sh || exit 1
TAG=pmc_r06_c4 PMC_BENCH="--config c4 --steps 1 --warmup 0 --no-cpu-baseline" bash tools/gpu_pmc_full.sh || exit 1
echo "pmc done"
