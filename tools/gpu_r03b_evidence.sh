#!/bin/bash
# GPU box, round 3 (second session): the default bench line (C3 with the C4 sub-line and the CPU baseline), then
# rocprof kernel traces and every PMC group for the configurations in $CONFIGS (tools/gpu_r03_profiles.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/${PROF_TAG:-prof_r03b}
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 400 python bench.py > gpurun_out/${PROF_TAG:-prof_r03b}/c3_bench.json 2> gpurun_out/${PROF_TAG:-prof_r03b}/c3_bench.err \
      || { echo "bench failed"; tail -5 gpurun_out/${PROF_TAG:-prof_r03b}/c3_bench.err; exit 1; }
  tail -c 400 gpurun_out/${PROF_TAG:-prof_r03b}/c3_bench.json
fi
PROF_TAG=${PROF_TAG:-prof_r03b} CONFIGS=${CONFIGS:-c3} bash tools/gpu_r03_profiles.sh
