#!/bin/bash
# GPU box (r06): C4 kernel stats with the merged shadow launch (RT_SHADOW_LAUNCH=2) beside the default (separate), to see
# where the merged schedule loses on C4.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 1 2; do
  RT_SHADOW_LAUNCH=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/c4m$m -o run -- \
      python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c4m$m.log 2>&1 || exit 1
  f=$(find gpurun_out/c4m$m -name "*kernel_trace.csv" | head -1)
  python3 tools/timeline.py "$f" --bucket-ms 5 > gpurun_out/c4m${m}_timeline.txt 2>&1
  echo "== RT_SHADOW_LAUNCH=$m"; head -14 gpurun_out/c4m${m}_timeline.txt
done
