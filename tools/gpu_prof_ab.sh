#!/bin/bash
# GPU box: rocprofv3 kernel stats of the default build and of every variant under lib/variants, for each
# bench.py argument set given as one quoted string; per-kernel totals side by side (tools/prof_cmp.py).
#   tools/gpu_prof_ab.sh "--config c3" "--config c4"
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pab
k=0
for args in "$@"; do
  k=$((k + 1))
  dirs=""
  for lib in buas-pathtracer_amd/lib/librt_mi355x.so buas-pathtracer_amd/lib/variants/*/librt_mi355x.so; do
    [ -f "$lib" ] || continue
    name=$(basename $(dirname $lib)); [ "$name" = lib ] && name=default
    out=gpurun_out/pab/${name}_$k
    RT_MI355X_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$out -o run -- \
        python3 bench.py $args --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --c4-steps 0 > $out.log 2>&1 \
        || { echo "$name [$args] failed"; tail -5 $out.log; exit 1; }
    dirs="$dirs $name=$out"
  done
  echo "== $args"
  python3 tools/prof_cmp.py $dirs
done
