#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group; never combined with tracing domains).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOTDIR=$(pwd)
export TMPDIR=/tmp
TAG=${TAG:-pmc}
mkdir -p gpurun_out/$TAG
if [ -n "$LIST" ]; then timeout -k 10 120 rocprofv3 -L > gpurun_out/$TAG/counters_list.txt 2>&1; echo "list rc=$?"; fi
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $ROOTDIR/gpurun_out/$TAG/pass$i -o run -- python3 $ROOTDIR/bench.py ${PMC_BENCH:---steps 1 --warmup 0 --spp 16 --no-cpu-baseline} > gpurun_out/$TAG/pass$i.log 2>&1
  rc=$?; echo "pass $i [$grp] rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
