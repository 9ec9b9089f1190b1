#!/bin/bash
# On the GPU box: bench every variant under buas-pathtracer_amd/lib/variants (plus the default build).
# BENCH_ARGS overrides the bench arguments. Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/variants
ARGS=${BENCH_ARGS:-"--spp 64 --steps 2 --warmup 1 --no-cpu-baseline"}
for lib in buas-pathtracer_amd/lib/librt_mi355x.so buas-pathtracer_amd/lib/variants/*/librt_mi355x.so; do
  [ -f "$lib" ] || continue
  name=$(basename $(dirname $lib)); [ "$name" = lib ] && name=default
  RT_MI355X_LIB=$PWD/$lib timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py $ARGS > gpurun_out/variants/$name.log 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -1 gpurun_out/variants/$name.log | python -c 'import json,sys
try:
  d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["stage_ms_per_step"])
except Exception as e: print("parse error", e)'
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
