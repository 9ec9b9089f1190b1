#!/bin/bash
# GPU box (r06): the sorted extension queue (rt_scene_config::sort_queue) -- equality tests, the
# lines-per-step probe (lib/variants/lines, tools/lines_probe.patch) unsorted and sorted, then the A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -k "sorted_queue or any_cadence or fused_drain or without_bvh" -v \
    --timeout 240 --timeout-method thread > gpurun_out/r06_sort_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r06_sort_tests.log | tail -12
[ $rc -ne 0 ] && exit $rc
for c in c3 c4; do
  for sq in 0 1; do
    RT_SORT_QUEUE=$sq RT_MI355X_LIB=$PWD/buas-pathtracer_amd/lib/variants/lines/librt_mi355x.so timeout -k 10 200 \
        python bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --c4-steps 0 > gpurun_out/r06_lines_${c}_$sq.log 2>&1 \
        || { echo "lines $c $sq failed"; tail -3 gpurun_out/r06_lines_${c}_$sq.log; exit 1; }
    echo "== $c sort_queue=$sq"; grep "lines probe" gpurun_out/r06_lines_${c}_$sq.log
  done
done
bash tools/gpu_ab_envs.sh "" "RT_SORT_QUEUE=1"
