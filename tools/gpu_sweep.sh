#!/bin/bash
# GPU box: the C3 bench once per "ENV ... -- bench args" variant (A/B on one box, no tests).
# usage: tools/gpu_sweep.sh "|" "RT_PARTITIONS=2|--pool 8388608" ...   (env|extra bench args)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
BASE=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu-baseline"}
i=0
for v in "$@"; do
  i=$((i+1))
  e=${v%%|*}; a=${v#*|}
  env $e timeout -k 10 200 python bench.py $BASE $a > gpurun_out/sw_$i.log 2>&1
  rc=$?; echo "== [$v] rc=$rc"; tail -1 gpurun_out/sw_$i.log | python -c 'import json,sys
try:
  d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["stage_ms_per_step"])
except Exception as e: print("parse error", e)'
  [ $rc -ne 0 ] && exit $rc
done
exit 0
