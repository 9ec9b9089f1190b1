#!/bin/bash
# GPU box: instruction-cache counters per kernel (one rocprofv3 --pmc pass; kernels serialized), C3 at 16 spp.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/icache
mkdir -p $OUT
timeout -s KILL 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES \
    --output-format csv -d $PWD/$OUT/p -o run -- python3 bench.py --spp 16 --steps 1 --warmup 0 --no-cpu-baseline \
    --c4-steps 0 > $OUT/run.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/run.log; exit 1; }
f=$(find $OUT/p -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")[:34]
    agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
for n, c in sorted(agg.items(), key=lambda x: -x[1].get("SQ_IFETCH", 0)):
    h, m = c.get("SQC_ICACHE_HITS", 0), c.get("SQC_ICACHE_MISSES", 0)
    print(f"{n:34s} ifetch/wave {c.get('SQ_IFETCH',0)/max(c.get('SQ_WAVES',1),1):9.1f}  icache hit {h/max(h+m,1):.4f}  misses {m:12.0f}  dup {c.get('SQC_ICACHE_MISSES_DUPLICATE',0):10.0f}")
PY
rm -rf $OUT/p
