#!/bin/bash
# GPU box: C4 (four unique 62.5k-triangle meshes, 14 MB of BVH and triangles) against C4i (one mesh
# instanced four times, 3.5 MB: fits an XCD's 4 MB L2): frame times, then the L2 hit rate of every
# kernel in one rocprofv3 --pmc pass each (TCC_HIT / TCC_MISS only).  Output under gpurun_out/loc/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/loc
mkdir -p $OUT
for rep in 1 2; do
  for c in c4 c4i; do
    timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --c4-steps 0 > $OUT/bench_${c}_$rep.log 2>&1 \
      || { echo "bench $c failed"; tail -5 $OUT/bench_${c}_$rep.log; exit 1; }
    echo "$c: $(tail -1 $OUT/bench_${c}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["closest_hit_rays"] if "closest_hit_rays" in d else "")')"
  done
done
for c in c4 c4i; do
  timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $PWD/$OUT/pmc_$c -o run -- \
      python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --c4-steps 0 > $OUT/pmc_$c.log 2>&1 \
      || { echo "pmc $c failed"; tail -5 $OUT/pmc_$c.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for c in ("c4", "c4i"):
    agg = collections.defaultdict(lambda: [0.0, 0.0])
    for f in glob.glob(f"gpurun_out/loc/pmc_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:28]
            i = 0 if r["Counter_Name"].startswith("TCC_HIT") else 1
            agg[k][i] += float(r["Counter_Value"])
    for k, (h, m) in sorted(agg.items(), key=lambda x: -sum(x[1])):
        if h + m > 0:
            print(f"{c:4s} {k:28s} L2 hit {h / (h + m):.3f}  requests {h + m:.3e}")
PY
