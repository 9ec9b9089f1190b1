#!/bin/bash
# GPU box: every PMC column of tools/pmc_summary.py, one rocprofv3 --pmc pass per counter group
# (never combined with tracing domains).  Counter names missing from `rocprofv3 -L` on this box
# are dropped from their group (listed in gpurun_out/$TAG/dropped.txt) instead of failing the pass.
#   TAG=pmc_r02 PMC_BENCH="--steps 1 --warmup 1 --spp 16 --no-cpu-baseline" tools/gpu_pmc_full.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOTDIR=$(pwd)
export TMPDIR=/tmp
TAG=${TAG:-pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1
echo "list rc=$?"
FILTER=1
grep -q "SQ_WAVES" $OUT/counters_list.txt || FILTER=0     # list unreadable: run the groups as given
GROUPS_DEFAULT=(
  "SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAVES"
  "SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES"
  "TCC_HIT_sum TCC_MISS_sum"
  "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
if [ $# -gt 0 ]; then GROUPS_RUN=("$@"); else GROUPS_RUN=("${GROUPS_DEFAULT[@]}"); fi
: > $OUT/dropped.txt
i=0
for grp in "${GROUPS_RUN[@]}"; do
  i=$((i+1))
  keep=""
  for c in $grp; do
    base=${c%_sum}
    if [ $FILTER = 0 ] || grep -qw -- "$c" $OUT/counters_list.txt || grep -qw -- "$base" $OUT/counters_list.txt; then keep="$keep $c"; else echo "$c" >> $OUT/dropped.txt; fi
  done
  if [ -z "$keep" ]; then echo "pass $i [$grp]: no counter available"; continue; fi
  timeout -s KILL 300 rocprofv3 --pmc $keep --output-format csv -d $ROOTDIR/$OUT/pass$i -o run -- python3 $ROOTDIR/bench.py ${PMC_BENCH:---steps 1 --warmup 0 --no-cpu-baseline} --c4-steps 0 > $OUT/pass$i.log 2>&1
  rc=$?; echo "pass $i [$keep] rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
