#!/bin/bash
# GPU-box sequence for a round checkpoint: parity tests -> full bench (C3) -> rocprofv3 kernel stats
# of the same workload -> PMC passes (FETCH_SIZE, WRITE_SIZE) for the HBM traffic of k_extend.
# Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOTDIR=$(pwd)
TAG=${TAG:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu_${TAG}.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 700 python bench.py ${BENCH_ARGS:---steps 3 --warmup 1} > gpurun_out/bench_${TAG}.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_${TAG}.log | cut -c1-1500
[ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp
PA=${PROF_ARGS:---steps 1 --warmup 1 --no-cpu-baseline}
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOTDIR/gpurun_out/prof_${TAG} -o run -- python3 $ROOTDIR/bench.py $PA > gpurun_out/prof_${TAG}.log 2>&1
rc=$?; echo "rocprof rc=$rc"
[ $rc -ne 0 ] && exit $rc
[ -n "$NO_PMC" ] && exit 0
mkdir -p gpurun_out/pmc_${TAG}
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 500 rocprofv3 --pmc $grp --output-format csv -d $ROOTDIR/gpurun_out/pmc_${TAG}/pass$i -o run -- python3 $ROOTDIR/bench.py $PA > gpurun_out/pmc_${TAG}/pass$i.log 2>&1 || { rc=$?; echo "pmc $grp rc=$rc"; exit $rc; }
  echo "pmc $grp ok"
done
exit 0
