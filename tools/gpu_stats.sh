cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in 1 0; do
RT_TOP_PROLOGUE=$v RT_DEBUG_TRAVERSAL=1 RT_MI355X_LIB=$PWD/buas-pathtracer_amd/lib/variants/stats/librt_mi355x.so timeout -k 10 300 python bench.py --spp 16 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/stats_$v.log 2>&1 || exit 1
grep 'step stats' gpurun_out/stats_$v.log | tail -2
done
