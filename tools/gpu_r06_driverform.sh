#!/bin/bash
# GPU box (r06 final tree): smoke() and the driver's own bench command (20 steps, 5 warm-up frames).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1 || { tail -5 gpurun_out/r06_smoke.log; exit 1; }
tail -1 gpurun_out/r06_smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_driverform.log 2>&1 || { tail -5 gpurun_out/r06_driverform.log; exit 1; }
tail -1 gpurun_out/r06_driverform.log | cut -c1-300
