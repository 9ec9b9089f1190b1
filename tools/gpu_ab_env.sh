#!/bin/bash
# GPU box: parity tests, then the bench once per environment setting (A/B).
# usage: tools/gpu_ab_env.sh "" "RT_PARTITIONS=1" "RT_PARTITIONS=3 RT_X=y" ...   ("" = as built)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E 'FAILED|ERROR|passed|failed' gpurun_out/pytest_gpu.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
ARGS=${BENCH_ARGS:-"--spp 64 --steps 2 --warmup 1 --no-cpu-baseline"}
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab_$i.log 2>&1
  rc=$?; echo "== [$v] rc=$rc"; tail -1 gpurun_out/ab_$i.log | python -c 'import json,sys
try:
  d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["stage_ms_per_step"], d["roofline"]["kernel"], d["roofline"]["concurrency"])
except Exception as e: print("parse error", e)'
  [ $rc -ne 0 ] && exit $rc
done
exit 0
