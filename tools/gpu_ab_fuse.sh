#!/bin/bash
# GPU box: the -m gpu suite (stops at the first failure), then an A/B of the fused drain on one box,
# alternating twice: this build, this build with RT_FUSE_PATHS=0 (fused drain off) and every variant
# under lib/variants; the full C3 frame and rank 0's share of an 8-rank frame; then a rocprof kernel
# trace of the share (tools/drain.py).  TAG=x bash tools/gpu_ab_fuse.sh [notests]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-fuse}
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
if [ "$1" != "notests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread \
      > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  grep -E "passed|failed" $OUT/pytest_gpu.log | tail -1
  cp gpurun_out/parity_report.json $OUT/ 2>/dev/null
fi
run() {   # name env lib mode
  local extra=""; [ $4 = s8 ] && extra="--shard-of 8"
  env $2 RT_MI355X_LIB=$PWD/$3 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline $extra \
      > $OUT/$1_$4.log 2>&1 || { echo "$1 $4 failed"; tail -20 $OUT/$1_$4.log; exit 1; }
  echo "$1 $4 $(tail -1 $OUT/$1_$4.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("rays_per_step", ""))')"
}
for rep in 1 2; do
  for mode in full s8; do
    run fused "RT_X=1" buas-pathtracer_amd/lib/librt_mi355x.so $mode
    run nofuse "RT_FUSE_PATHS=0" buas-pathtracer_amd/lib/librt_mi355x.so $mode
    for lib in buas-pathtracer_amd/lib/variants/*/librt_mi355x.so; do
      [ -f "$lib" ] || continue
      run $(basename $(dirname $lib)) "RT_X=1" $lib $mode
    done
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $PWD/$OUT/prof_s8 -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --shard-of 8 > $OUT/prof_s8.log 2>&1 \
    || { echo "rocprof failed"; tail -20 $OUT/prof_s8.log; exit 1; }
echo done
