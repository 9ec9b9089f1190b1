#!/usr/bin/env python3
"""Benchmark: Mrays/s (+ samples/s/GPU) of the MI355X wavefront path tracer.

BASELINE.json metric: "Mrays/s + samples/s/GPU at 1080p 256spp; 1/2/4/8-GPU
scaling".  The default workload is configs[2] (C3: Cornell box + ~70k-tri
synthetic mesh with SAH BVH + synthetic 2048x1024 HDR environment + NEE + RR,
1920x1080, 256 spp, max depth 12) — the 1-GPU configuration the metric is
quoted on.  One step = one full frame of that workload: this rank's share of
the frame integrated into an fp32 float4 accumulation buffer already resident
in HBM, plus (N > 1) the RCCL sum-reduce of the framebuffer over xGMI.  A
rank's share is, by default, sample passes [spp*r/N, spp*(r+1)/N) of every
tile (--shard-mode passes: equal cost per rank whatever the content); with
--shard-mode tiles it is the tiles t % N (the reference's 64x64 tile queue
dealt round robin).  Strong scaling: the frame is fixed, the work is split
over the ranks.  The JSON's `c4` object times the north star's own scene
(C4) on the same ranks.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3] [--no-cpu-baseline]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
    python -m torch.distributed.run --nproc-per-node 1 ... bench.py --force-dist   (the RCCL path at one rank)

Rank 0 prints ONE JSON line.  `roofline` is for the dominant kernel: the stage
with the most GPU time in the timed region (k_shade on C3), algorithmic bytes =
its SURVEY.md §8(d) bytes per unit (BYTES_PER_UNIT) x units per launch / mean
launch time, measured with HIP events on the stream of the partition that
launched it.  Four partitions run concurrently, so the launch
time includes shared GPU time: `concurrency` gives the mean number of kernels in
flight, `isolated` the serialized figures from the rocprofv3 --pmc runs, and
`pipeline` the whole-frame figure of SURVEY.md §8(d) (152 B per ray + 144 B per
sample over wall time), and `traversal` the trace kernels' step fetches (128 B per
step, the timed frames' own rt_stats::trace_steps) over their launch time.  The
frame's TraversalStats (rt_stats::traversal, the reference's per-frame counters)
are in `traversal_stats`.  `cpu_baseline` is the CPU restatement (oracle/,
reference-stream RNG, 64x64 tile queue) timed on this box's cores over a
bounded sample of the same workload.
"""
import argparse
import ctypes as C
import importlib.util
import json
import os
import sys
import time

# dmabuf IPC for RCCL and cross-process CUDA tensors (the host driver has no legacy IPC); it must be in
# the environment before torch (and HIP) initialise
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

ROOT = os.path.dirname(os.path.abspath(__file__))
METRIC = "Mrays/s + samples/s/GPU at 1080p 256spp; 1/2/4/8-GPU scaling"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E, MI355X_MICROARCH.md chip table
L2_PEAK_GBS = 16800.0          # rows gathered from the XCDs' L2, chip-wide (MI355X_MICROARCH.md, lower bound)
STAGES = ["generate", "extend", "shade", "connect", "splat", "resolve"]
# "extend" is the trace launch of an iteration's extension rays; with the merged shadow launch (r06,
# rt_scene_config::shadow_launch: a rank's share of a multi-GPU frame) it also traces the previous
# iteration's shadow rays and "connect" (RT_KERNEL_CONNECT) has no launches; otherwise "connect" is the
# separate shadow launch
KERNEL = {"generate": "k_generate", "extend": "k_trace", "shade": "k_shade", "connect": "k_trace_shadow",
          "splat": "k_splat", "resolve": "k_resolve"}
# Algorithmic HBM bytes per unit of work, with the unit each launch processes:
#   generate: a new path's ray (32 B) + path state (48 B) written                  per sample
#   extend:   the queued record (o|slot, d|t, 1/d: 48 B) in, the hit (20 B) out    per traced closest-hit ray
#   shade:    hit 16 + state 48 in, state 48 + next ray 32 + shadow ray 48 out    per closest-hit query shaded
#   connect:  the shadow record (48 B) + contribution (16 B) in                   per traced shadow ray
#   splat:    path state 48 B in, the 16 B sample record out                      per sample
BYTES_PER_UNIT = {"generate": 80, "extend": 68, "shade": 192, "connect": 64, "splat": 64}


def stage_work(stage, samples, closest, traced, traced_sh, merged):
    """(units, algorithmic bytes) of a stage's launches over some frames.  merged (no separate shadow
    launches): the trace launch ("extend") does the traced closest-hit rays (68 B) and the traced shadow
    rays (64 B)."""
    if stage == "extend" and merged:
        return traced + traced_sh, BYTES_PER_UNIT["extend"] * traced + BYTES_PER_UNIT["connect"] * traced_sh
    if stage == "extend":
        return traced, BYTES_PER_UNIT["extend"] * traced
    units = {"generate": samples, "shade": closest, "connect": traced_sh, "splat": samples}[stage]
    return units, BYTES_PER_UNIT[stage] * units
# whole-pipeline figure of SURVEY.md §8(d): B_alg = 152 B per ray + 144 B per sample
PIPE_BYTES_PER_RAY, PIPE_BYTES_PER_SAMPLE = 152, 144
CONFIGS = {
    "c1": dict(preset="c1", w=512, h=512),
    "c2": dict(preset="c2", w=1920, h=1080),
    "c3": dict(preset="c3", w=1920, h=1080),
    "c4": dict(preset="c4", w=1920, h=1080),
    "c4i": dict(preset="c4i", w=1920, h=1080),     # C4 with one mesh instanced 4 times (the reference's scene)
    "c5": dict(preset="c5", w=3840, h=2160),
}


def import_package():
    name = "buas_pathtracer_amd"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(
        name, os.path.join(ROOT, "buas-pathtracer_amd", "__init__.py"),
        submodule_search_locations=[os.path.join(ROOT, "buas-pathtracer_amd")])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def host_cores():
    """The cores this process may run on: the affinity mask, capped by the cgroup CPU quota (a GPU
    box shows the whole machine in os.cpu_count() but grants each GPU a share of it)."""
    nproc = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    cores = affinity if quota is None else max(1, min(affinity, int(quota + 0.5)))
    return {"cores": cores, "nproc": nproc, "affinity": affinity, "cgroup_quota_cores": quota}


def cpu_baseline(rt, cfg, spp_override, seconds_budget=15.0):
    """Oracle (C restatement, reference-stream RNG, tile queue) on a bounded tile sample, at the
    box's core count N and at the reference's own 1.25 N worker threads (RT/raytracer.cpp:1580-1592)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import oracle_binding as ob
    lib = ob.load()
    hc = host_cores()
    threads = int(os.environ.get("RT_CPU_THREADS", hc["cores"]))
    scene, cam, st, fc, post = rt.load_preset(cfg["preset"], cfg["w"], cfg["h"], asset_dir=None)
    if spp_override:
        st.samples_per_pixel = spp_override
    w, h = cfg["w"], cfg["h"]
    tcx, tcy = (w + 63) // 64, (h + 63) // 64
    total_tiles = tcx * tcy
    # calibrate with one tile at the full spp, then size the sample to the budget
    accum = np.zeros((h, w, 4), np.float32)
    buf = rt.abi.AccumulationBuffer(w, h, 0, accum.ctypes.data_as(C.POINTER(C.c_float)))
    desc = scene.desc()

    def run(tiles, nthreads):
        arr = (C.c_uint32 * len(tiles))(*tiles)
        stats = rt.abi.Stats()
        t0 = time.perf_counter()
        err = lib.oracle_render_tiles(C.byref(desc), C.byref(cam), C.byref(st), C.byref(fc), 64, 64, 0,
                                      1, nthreads, len(tiles), arr, C.byref(buf), C.byref(stats))
        assert err == 0
        return time.perf_counter() - t0, stats

    mid = [total_tiles // 2 + tcx // 2]
    t1, _ = run(mid, 1)
    n_tiles = max(threads, min(total_tiles, int(seconds_budget * threads / max(t1, 1e-3))))
    n_tiles = max(1, (n_tiles // threads) * threads) if n_tiles >= threads else n_tiles
    step = max(1, total_tiles // n_tiles)
    tiles = [(k * step + step // 2) % total_tiles for k in range(n_tiles)]
    dt, stats = run(tiles, threads)
    rays = stats.closest_hit_rays + stats.shadow_rays
    # the reference's worker count, 1.25 x the cores (RT/raytracer.cpp:1588), on the same tiles
    t125 = max(1, int(threads * 1.25))
    dt125, stats125 = run(tiles, t125)
    rays125 = stats125.closest_hit_rays + stats125.shadow_rays
    return {"value": rays / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "samples_per_s": stats.samples / dt,
            "host": hc,
            "threads_1p25": {"threads": t125, "value": rays125 / dt125 / 1e6, "samples_per_s": stats125.samples / dt125,
                             "seconds": round(dt125, 2)},
            "sample": f"{n_tiles} of {total_tiles} 64x64 tiles (evenly spaced) of the same {w}x{h} "
                      f"{st.samples_per_pixel}spp frame, reference-stream RNG, {threads} threads "
                      f"(the box's cores: affinity {hc['affinity']}, cgroup quota {hc['cgroup_quota_cores']}, "
                      f"nproc {hc['nproc']}), {dt:.1f} s, {rays} rays; again at {t125} threads"}


def pmc_figures(tj, kname, units_per_frame, alg, launches_per_frame):
    """The serialized (rocprofv3 --pmc) figures of kernel `kname` from one configuration's entry of
    profiles/traffic.json, normalized per frame over the same frame as the algorithmic bytes: the sum
    of the isolated durations and of the HBM bytes over ALL of the kernel's dispatches in one frame
    (the early exits after a partition's end included) against `alg`, the algorithmic bytes of one
    frame's units.  `traffic` per launch divides the frame's counter bytes by the launches the units are
    averaged over (the event-timed ones), so it is comparable with `achieved`.  None when the entry
    is missing or was measured on a frame of another size (units per frame off by more than 10 %)."""
    ent = (tj or {}).get("kernels", {}).get(kname)
    frames = (tj or {}).get("frames_per_pass")
    upf = ((tj or {}).get("units_per_frame") or {}).get(kname)
    if not ent or not frames or not upf or not units_per_frame:
        return None
    if abs(upf / units_per_frame - 1.0) > 0.1:
        return None
    disp = ent["dispatches"] / frames
    iso_s = ent["isolated_mean_us"] * 1e-6 * disp
    hbm = ent["hbm_bytes_per_launch"] * disp
    gbs = alg / iso_s / 1e9
    return {"isolated": {"frame_ms": round(iso_s * 1e3, 3), "dispatches_per_frame": round(disp, 1),
                         "mean_dispatch_ms": round(ent["isolated_mean_us"] / 1e3, 4),
                         "alg_bytes_per_frame": round(alg), "achieved": round(gbs, 1),
                         "frac": round(gbs / HBM_PEAK_GBS, 4), "source": tj.get("source"),
                         "normalization": "per frame: the algorithmic bytes of one frame's units / the sum of "
                                          "the kernel's serialized dispatch durations in one frame"},
            "traffic": round(hbm / max(launches_per_frame, 1e-9)),
            "traffic_per_frame": round(hbm), "traffic_ratio": round(hbm / alg, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--spp", type=int, default=0, help="override samples per pixel (0 = config's)")
    ap.add_argument("--width", type=int, default=0)
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--pool", type=int, default=0, help="in-flight path pool size (0 = default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--shard-index", type=int, default=0, help="with --shard-of: which rank's share (diagnostic)")
    ap.add_argument("--shard-mode", choices=["tiles", "passes"], default="passes",
                    help="what a rank's share of the frame is: a range of sample passes over every tile (default: "
                         "equal cost per rank whatever the content) or tiles t %% N (DESIGN.md section 7)")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="diagnostic (1 process): render only rank 0's tiles of an N-rank frame, to size the "
                         "per-rank work of the N-GPU strong-scaling run; not a bench line")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--env-sampling", type=int, default=0,
                    help="1: environment-map NEE (rt_set_env_sampling; beyond the reference's estimator)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl (= RCCL over xGMI, the product path) or gloo (framebuffer reduced through host "
                         "memory: lets several ranks share one GPU in the tests)")
    ap.add_argument("--c4-steps", type=int, default=5,
                    help="also time the north star's own scene (C4, 1080p 256 spp) for this many frames "
                         "after one warm-up frame, same ranks and sharding (0 = skip)")
    ap.add_argument("--dump-frame", default="",
                    help="rank 0 saves the accumulated frame of the last timed step (.npy; tests)")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the distributed path (process group, the framebuffer reduce into rank 0, the "
                         "all-reduces of the totals) even with one rank, e.g. RCCL at --nproc-per-node 1")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1 or args.force_dist
    # one GPU per rank; ranks beyond the visible GPUs share them (gloo tests on a 1-GPU box)
    device = local_rank % max(1, torch.cuda.device_count())
    if distributed:
        torch.cuda.set_device(device)
        dist.init_process_group(args.dist_backend, rank=rank, world_size=world)
    torch.cuda.set_device(device)
    # the ray / time totals go through the backend's own memory (gloo reduces host tensors)
    red_dev = "cpu" if args.dist_backend == "gloo" else f"cuda:{device}"

    rt = import_package()

    def traffic_cfg(name):
        """profiles/traffic.json's entry for one bench configuration (tools/pmc_summary.py --traffic)."""
        try:
            with open(args.traffic_json) as f:
                return json.load(f).get("configs", {}).get(name)
        except (OSError, ValueError):
            return None
    cfg = dict(CONFIGS[args.config])
    if args.width:
        cfg["w"] = args.width
    if args.height:
        cfg["h"] = args.height
    w, h = cfg["w"], cfg["h"]
    # Synthetic assets go through their files (the OBJ / RGBE parsers) on one rank only; ranks
    # started together build them in memory, so none can read another's file mid-write.
    asset_dir = None
    if world == 1:
        import tempfile
        asset_dir = os.path.join(tempfile.gettempdir(), f"rt_assets_{os.getuid()}")
        os.makedirs(asset_dir, exist_ok=True)
    shard_mode = rt.abi.RT_SHARD_PASSES if args.shard_mode == "passes" else rt.abi.RT_SHARD_TILES
    stream = torch.cuda.current_stream(device)
    from buas_pathtracer_amd.sharding import render_frame_sharded, timing_summary

    def setup(name, fw, fh, adir):
        scene, cam, st, fc, post = rt.load_preset(CONFIGS[name]["preset"], fw, fh, asset_dir=adir)
        dev = rt.DeviceScene(scene, device)
        # per-scene settings (rt_scene_config): this scene's shard mode, pool and environment NEE
        dev.configure(shard_mode=shard_mode, path_pool=args.pool, env_sampling=1 if args.env_sampling else 0)
        accum = torch.zeros((fh, fw, 4), dtype=torch.float32, device=f"cuda:{device}")
        scratch = torch.zeros_like(accum) if distributed else None

        def render_shard(shard_index, shard_count, buf):
            return dev.render_device(cam, st, fc, fw, fh, buf.data_ptr(), stream=stream.cuda_stream,
                                     shard_index=shard_index, shard_count=shard_count)

        def step(timing=None):
            accum.zero_()
            if args.shard_of > 1:                          # diagnostic: one rank's share of an N-rank frame
                t0 = time.perf_counter()
                s = render_shard(args.shard_index, args.shard_of, accum)
                if timing is not None:
                    timing.setdefault("render_s", []).append(time.perf_counter() - t0)
                return s
            # this rank's share into a zeroed frame buffer, the RCCL sum-reduce of it over xGMI into
            # rank 0, which adds it to its accumulation buffer
            return render_frame_sharded(render_shard, accum, rank, world, scratch=scratch, reduce=distributed,
                                        timing=timing)
        return scene, dev, st, post, accum, step

    scene, dev, st, post, accum, step = setup(args.config, w, h, asset_dir)
    if args.spp:
        st.samples_per_pixel = args.spp

    # Warm-up frames time every stage (HIP events around each launch); the timed region
    # then records events for the dominant stage only, since each event pair is a queue
    # marker that costs the other launches ~0.5 % of the frame (2.4 % for all stages).
    rt.lib().rt_set_profiling(1)
    wms = [0.0] * 6
    wl = [0] * 6                    # warm-up launches per stage, and the rays the trace stages got
    wtraced = [0, 0]
    # The stage statistics cover the warm-up frames since the last change of the shadow launch: a whole
    # frame's auto policy reads the scene's previous frame (rt_scene_config::shadow_launch), so a scene's
    # first frame may trace its shadow rays in another launch than the frames after it.
    nwf, wmode = 0, None
    for _ in range(args.warmup):
        s = step()
        if s.shadow_launch != wmode:
            wms, wl, wtraced, nwf, wmode = [0.0] * 6, [0] * 6, [0, 0], 0, s.shadow_launch
        nwf += 1
        for k in range(6):
            wms[k] += s.kernel_ms[k]
            wl[k] += s.kernel_launches[k]
        wtraced[0] += s.traced_rays[0]
        wtraced[1] += s.traced_rays[1]
    if nwf:
        wms = [x / nwf for x in wms]
    torch.cuda.synchronize(device)
    if args.warmup:
        dom_stage = max(range(5), key=lambda k: wms[k])
        rt.lib().rt_set_profiling_stages(1 << dom_stage)
    if os.environ.get("RT_BENCH_NO_STAGE_EVENTS"):
        rt.lib().rt_set_profiling(0)
    closest = shadow = samples = traced = traced_sh = 0
    separate = 0                     # timed frames with the separate shadow launch (rt_stats::shadow_launch)
    steps_k = [0, 0]                 # trace steps (rt_stats::trace_steps) of the timed frames, per kind
    trav = [dict.fromkeys(rt.abi.TRAVERSAL_FIELDS, 0) for _ in range(2)]
    kms = [0.0] * 6
    kl = [0] * 6
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(device)
    timing = {}                      # per-step render / reduce times of this rank (rank diagnostics)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        s = step(timing)
        closest += s.closest_hit_rays
        shadow += s.shadow_rays
        samples += s.samples
        traced += s.traced_rays[0]
        traced_sh += s.traced_rays[1]
        separate += s.shadow_launch == rt.abi.RT_SHADOW_LAUNCH_SEPARATE
        for k in range(2):
            steps_k[k] += s.trace_steps[k]
            for f in rt.abi.TRAVERSAL_FIELDS:
                trav[k][f] += getattr(s.traversal[k], f)
        for k in range(6):
            kms[k] += s.kernel_ms[k]
            kl[k] += s.kernel_launches[k]
    torch.cuda.synchronize(device)
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    rt.lib().rt_set_profiling(0)

    totals = torch.tensor([closest, shadow, samples, traced, traced_sh] + steps_k +
                          [trav[k][f] for k in range(2) for f in rt.abi.TRAVERSAL_FIELDS],
                          dtype=torch.float64, device=red_dev)
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
    if distributed:
        dist.all_reduce(totals, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    # Per-rank diagnostics (N > 1): each rank's frame (render) times, its framebuffer reduce times and
    # its samples, gathered to rank 0 -- so a scaling shortfall reads as imbalance, tail or reduce.
    ranks_info = None
    tsum = timing_summary(timing)
    if distributed and tsum["render_ms"]:
        fr, rd = tsum["render_ms"], tsum["reduce_ms"]
        row = [min(fr), sum(fr) / len(fr), max(fr), (sum(rd) / len(rd)) if rd else 0.0, max(rd) if rd else 0.0,
               float(samples), 1e3 * elapsed / args.steps]
        table = torch.zeros((world, len(row)), dtype=torch.float64, device=red_dev)
        table[rank] = torch.tensor(row, dtype=torch.float64, device=red_dev)
        dist.all_reduce(table, op=dist.ReduceOp.SUM)
        rows = table.cpu().tolist()
        ranks_info = {
            "world_size": dist.get_world_size(), "backend": dist.get_backend(),
            "device_count": torch.cuda.device_count(),
            "per_rank": [{"rank": r, "frame_ms": {"min": round(x[0], 3), "mean": round(x[1], 3), "max": round(x[2], 3)},
                          "reduce_ms": {"mean": round(x[3], 3), "max": round(x[4], 3)},
                          "samples": int(x[5]), "step_ms": round(x[6], 3)} for r, x in enumerate(rows)],
            "frame_ms_max_over_ranks": round(max(x[2] for x in rows), 3),
            "frame_ms_mean_over_ranks": round(sum(x[1] for x in rows) / world, 3),
            "reduce_ms_mean_over_ranks": round(sum(x[3] for x in rows) / world, 3),
            "note": "frame_ms: host wall time of rt_render_device per timed step (it returns once the rank's share "
                    "is done on the GPU); reduce_ms: HIP events around the RCCL reduce on the render stream (gloo: "
                    "host time of the staged host reduce); step_ms: the rank's own timed-region time per step"}
    tl = [float(x) for x in totals.tolist()]
    closest_all, shadow_all, samples_all, traced_all, traced_sh_all = tl[:5]
    nf = len(rt.abi.TRAVERSAL_FIELDS)
    trav_all = [{f: int(tl[7 + k*nf + i]) for i, f in enumerate(rt.abi.TRAVERSAL_FIELDS)} for k in range(2)]
    elapsed = float(tmax.item())
    if args.dump_frame and rank == 0:
        import numpy as np
        np.save(args.dump_frame, accum.cpu().numpy())

    # The north star's own scene (BASELINE configs[3], C4: ~250k triangles, 1080p, 256 spp), timed on
    # the same ranks with the same sharding: one warm-up frame, then --c4-steps frames.
    c4 = None
    if args.c4_steps > 0 and args.config != "c4" and args.shard_of <= 1:
        c4scene, c4dev, c4st, _, c4acc, c4step = setup("c4", CONFIGS["c4"]["w"], CONFIGS["c4"]["h"], asset_dir)
        # C4's roofline is the trace launch's (k_trace, the kernel with the most GPU time there): HIP
        # events around the extend launches only, in the warm-up and the timed frames
        ext = STAGES.index("extend")
        rt.lib().rt_set_profiling_stages(1 << ext)
        c4step()
        torch.cuda.synchronize(device)
        if distributed:
            dist.barrier()
        c0 = time.perf_counter()
        cr = [0, 0, 0]
        cx = [0.0, 0, 0, 0, 0, 0]       # trace launch: event ms, launches, traced closest / shadow rays, trace steps,
                                        # frames with the separate shadow launch
        for _ in range(args.c4_steps):
            cs = c4step()
            cr[0] += cs.closest_hit_rays
            cr[1] += cs.shadow_rays
            cr[2] += cs.samples
            cx[0] += cs.kernel_ms[ext]
            cx[1] += cs.kernel_launches[ext]
            cx[2] += cs.traced_rays[0]
            cx[3] += cs.traced_rays[1]
            cx[5] += cs.shadow_launch == rt.abi.RT_SHADOW_LAUNCH_SEPARATE
            cx[4] += cs.trace_steps[0] + (cs.trace_steps[1] if not cx[5] else 0)
        torch.cuda.synchronize(device)
        if distributed:
            dist.barrier()
        rt.lib().rt_set_profiling(0)
        ct = torch.tensor([time.perf_counter() - c0], dtype=torch.float64, device=red_dev)
        crt = torch.tensor(cr, dtype=torch.float64, device=red_dev)
        if distributed:
            dist.all_reduce(crt, op=dist.ReduceOp.SUM)
            dist.all_reduce(ct, op=dist.ReduceOp.MAX)
        c4dev.close()
        cel = float(ct.item())
        c4_rays = float(crt[0]) + float(crt[1])
        c4 = {"workload": f"c4: c4 {CONFIGS['c4']['w']}x{CONFIGS['c4']['h']} {c4st.samples_per_pixel}spp "
                          f"depth {c4st.max_bounce_count} (~250k triangles, four meshes, nested dielectrics)",
              "steps": args.c4_steps, "warmup": 1, "ms_per_step": round(1e3 * cel / args.c4_steps, 3),
              "value": round(c4_rays / cel / 1e6, 3), "unit": "Mrays/s",
              "samples_per_s": round(float(crt[2]) / cel, 1),
              "samples_per_s_per_gpu": round(float(crt[2]) / cel / world, 1),
              "closest_hit_rays": int(crt[0]), "shadow_rays": int(crt[1])}
        # rank 0's trace launch (k_trace): 68 B per traced closest-hit ray + 64 B per traced shadow ray (SURVEY.md
        # section 8(d)) over the launches' HIP-event time; the serialized figures and counter traffic from
        # profiles/traffic.json's c4 entry (same frame size only); the step fetches (128 B per trace step, the
        # frames' own counts) against the L2 rate
        if cx[1] and cx[0] > 0:
            n = args.c4_steps
            mean_s = cx[0] / cx[1] / 1e3
            u4, b4 = stage_work("extend", 0, 0, cx[2], cx[3], merged=not cx[5])
            gbs = b4 / cx[1] / mean_s / 1e9
            tgbs = 128.0 * cx[4] / cx[1] / mean_s / 1e9
            k4 = "k_trace_ext" if cx[5] else "k_trace"
            pmc4 = pmc_figures(traffic_cfg("c4"), k4, u4 / n, b4 / n, cx[1] / n)
            c4["roofline"] = {"bound": "hbm", "kernel": k4, "bytes_per_unit": round(b4 / max(u4, 1), 2),
                              "units_per_launch": round(u4 / cx[1], 1), "mean_launch_ms": round(mean_s * 1e3, 4),
                              "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": round(gbs / HBM_PEAK_GBS, 6),
                              "traffic": pmc4["traffic"] if pmc4 else None,
                              "traffic_ratio": pmc4["traffic_ratio"] if pmc4 else None,
                              "isolated": pmc4["isolated"] if pmc4 else None,
                              "traversal": {"bytes_per_step": 128, "steps_per_ray": round(cx[4] / max(u4, 1), 3),
                                            "achieved": round(tgbs, 1), "peak": L2_PEAK_GBS,
                                            "frac": round(tgbs / L2_PEAK_GBS, 4)},
                              "timing": "HIP events around rank 0's trace launches in the timed C4 frames "
                                        "(four partitions share the GPU); units: traced closest-hit + shadow rays"}

    if rank == 0:
        rays = closest_all + shadow_all
        mrays = rays / elapsed / 1e6
        # Roofline of the dominant kernel (most event-timed GPU time in the timed region) on rank 0.
        # Each stage's begin/end HIP events are recorded on the stream of the partition that
        # launched it, so with 4 partitions in flight a launch's duration includes the GPU
        # time it shares with the other partitions' kernels: `concurrency` says how many
        # kernels ran at once on average, and `isolated` gives the serialized figures
        # (rocprofv3 --pmc runs, profiles/traffic.json) for the same kernel.
        merged = not separate                       # the frames' shadow rays rode in the trace launch
        if not merged:
            KERNEL.update({"extend": "k_trace_ext", "connect": "k_trace_shadow"})
        work = {k: stage_work(k, samples, closest, traced, traced_sh, merged) for k in BYTES_PER_UNIT}
        dom = max(BYTES_PER_UNIT, key=lambda k: kms[STAGES.index(k)])     # the only stage timed (warm-up > 0)
        di = STAGES.index(dom)
        mean_launch_s = (kms[di] / 1e3) / max(kl[di], 1)
        units_per_launch = work[dom][0] / max(kl[di], 1)
        alg_bytes = work[dom][1] / max(kl[di], 1)
        achieved = alg_bytes / mean_launch_s / 1e9 if mean_launch_s > 0 else 0.0
        pmc = pmc_figures(traffic_cfg(args.config), KERNEL[dom], work[dom][0] / args.steps, work[dom][1] / args.steps,
                          kl[di] / args.steps)
        traffic = pmc["traffic"] if pmc else None
        isolated = pmc["isolated"] if pmc else None
        # Traversal kernels are bound by dependent L2 / Infinity Cache fetches, not HBM: their second
        # figure is the bytes their steps fetch -- every step loads one 128-byte round per lane (a BVH4
        # node, two triangles or a leaf record) -- counted in the timed frames by the kernels themselves
        # (rt_stats::trace_steps, rank 0), over the launches' HIP-event time in the warm-up frames (every
        # stage timed there; the frames are identical), against the L2 gather rate (MI355X_MICROARCH.md,
        # rows shared by every workgroup: 16.8-18.8 TB/s).  Reported for both trace kernels.
        traversal = None
        if args.warmup and (wmode == rt.abi.RT_SHADOW_LAUNCH_MERGED) == merged:
            traversal = {"peak": L2_PEAK_GBS, "unit": "GB/s", "bytes_per_step": 128,
                         "source": "rt_stats::trace_steps of the timed frames (counted on the device; the trace launches' "
                                   "own steps, closest-hit and shadow, the fused drain's left out)",
                         "timing": "warm-up frames, HIP events on each partition's stream (shared GPU)"}
            # the trace launch (merged: both kinds of ray), and the separate shadow launch when there is one
            kinds = [("extend", "k_trace", traced + traced_sh if merged else traced,
                      steps_k[0] + steps_k[1] if merged else steps_k[0])]
            if not merged:
                kinds[0] = ("extend", "k_trace_ext", traced, steps_k[0])
                kinds.append(("connect", "k_trace_shadow", traced_sh, steps_k[1]))
            for stage, kname, rays, ksteps in kinds:
                k = STAGES.index(stage)
                if not wl[k] or wms[k] <= 0 or not rays:
                    continue
                launches = wl[k] / nwf                             # per frame
                steps = ksteps / args.steps                         # per frame
                tb = 128.0 * steps / launches
                mean_s = wms[k] / launches / 1e3
                t_gbs = tb / mean_s / 1e9
                traversal[kname] = {"rays_per_launch": round(rays / args.steps / launches),
                                    "steps_per_ray": round(ksteps / rays, 3),
                                    "bytes_per_launch": round(tb), "mean_launch_ms": round(mean_s * 1e3, 4),
                                    "achieved": round(t_gbs, 1), "frac": round(t_gbs / L2_PEAK_GBS, 4)}
        ref = wms if args.warmup else [x / args.steps for x in kms]        # all stages: warm-up frames
        concurrency = sum(ref[:5]) / (elapsed * 1e3 / args.steps) if elapsed > 0 else 0.0
        pipe_bytes = PIPE_BYTES_PER_RAY * (closest + shadow) + PIPE_BYTES_PER_SAMPLE * samples
        pipe_gbs = pipe_bytes / elapsed / 1e9
        # output pass on the resolved frame: k_post, 16 B read + 4 B written per pixel
        bgra = torch.empty((h, w), dtype=torch.int32, device=f"cuda:{device}")
        pcall = lambda: rt.lib().rt_postprocess_device(device, C.c_void_p(accum.data_ptr()), w, h, C.byref(post), 0,
                                                       C.c_void_p(bgra.data_ptr()), C.c_void_p(stream.cuda_stream))
        for _ in range(3):
            assert pcall() == 0, rt.lib().rt_last_error()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        post_ms = []
        for _ in range(20):
            ev[0].record(stream)
            assert pcall() == 0
            ev[1].record(stream)
            ev[1].synchronize()
            post_ms.append(ev[0].elapsed_time(ev[1]))
        post_ms = sorted(post_ms)[len(post_ms) // 2]
        post_gbs = 20.0 * w * h / (post_ms * 1e-3) / 1e9
        postprocess = {"kernel": "k_post", "ms": round(post_ms, 4), "achieved_GBps": round(post_gbs, 1),
                       "frac_of_hbm_peak": round(post_gbs / HBM_PEAK_GBS, 4), "bytes_per_pixel": 20,
                       "note": "median of 20 calls, HIP events on the render stream around each call "
                               "(includes launch latency); rocprof gives the kernel alone"}
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(rt, cfg, args.spp, args.cpu_seconds)
        parallelism = (f"{args.shard_mode}%{args.shard_of} (rank {args.shard_index} only, diagnostic)"
                       if args.shard_of > 1 else f"{args.shard_mode}%{world}" +
                       (f"+{'rccl' if args.dist_backend == 'nccl' else 'gloo'}_reduce" if distributed else ""))
        out = {
            "metric": METRIC,
            "value": round(mrays, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "samples_per_s": round(samples_all / elapsed, 1),
            "samples_per_s_per_gpu": round(samples_all / elapsed / world, 1),
            "closest_hit_rays": int(closest_all),
            "shadow_rays": int(shadow_all),
            # the rays handed to the BVH traversal kernels (closest, shadow); the rest were settled by the
            # planes / top-level prologue where they were made
            "traced_rays": [int(traced_all), int(traced_sh_all)],
            # rank 0's units of work per frame per kernel (tools/pmc_summary.py --traffic keeps them with
            # the PMC figures, which bench.py uses only for frames of the same size)
            "units_per_frame": {KERNEL[k]: round(work[k][0] / args.steps, 1)
                                for k in ("generate", "extend", "shade") + (() if merged else ("connect",))},
            "shadow_launch": "merged into the trace launch" if merged else "separate",
            "config": {"workload": f"{args.config}: {cfg['preset']} {w}x{h} {st.samples_per_pixel}spp "
                                   f"depth {st.max_bounce_count}" + (" env-sampling" if args.env_sampling else ""),
                       "width": w, "height": h,
                       "spp": st.samples_per_pixel, "max_depth": st.max_bounce_count,
                       "parallelism": parallelism,
                       "shard_mode": args.shard_mode,
                       "shard_modes": "passes: rank r renders sample passes [spp*r/N, spp*(r+1)/N) of every tile "
                                      "(default, equal cost per rank); tiles: tile t on rank t % N (the north "
                                      "star's wording, --shard-mode tiles); both sum to the same frame "
                                      "(DESIGN.md section 7)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
                         "kernel": KERNEL[dom], "bytes_per_unit": round(alg_bytes / max(units_per_launch, 1e-9), 2),
                         "units_per_launch": round(units_per_launch, 1),
                         "mean_launch_ms": round(mean_launch_s * 1e3, 4),
                         "traffic_ratio": pmc["traffic_ratio"] if pmc else None,
                         "traffic_per_frame": pmc["traffic_per_frame"] if pmc else None,
                         "concurrency": round(concurrency, 2), "isolated": isolated, "traversal": traversal,
                         "pipeline": {"bytes": pipe_bytes, "achieved": round(pipe_gbs, 1),
                                      "frac": round(pipe_gbs / HBM_PEAK_GBS, 4),
                                      "formula": "152 B x (closest + shadow rays) + 144 B x samples, rank 0, / wall time"}},
            "stage_ms_per_step": {n: round((wms[i] if args.warmup else kms[i] / args.steps), 2) for i, n in
                                  enumerate(STAGES)},
            "stage_ms_note": ("HIP-event time per stage summed over its launches, from the warm-up frames "
                              "(4 partitions overlap, so the sum exceeds ms_per_step)"),
            # the reference's per-frame TraversalStats (RT/intersection.h:33-40), counted on the device in
            # this library's walk and BVH4 units (include/rt_abi.h), per frame, all ranks
            "traversal_stats": {"per_frame": {f: (trav_all[0][f] + trav_all[1][f]) // args.steps
                                              for f in rt.abi.TRAVERSAL_FIELDS},
                                "closest": {f: v // args.steps for f, v in trav_all[0].items()},
                                "shadow": {f: v // args.steps for f, v in trav_all[1].items()}},
            "c4": c4,
            "ranks": ranks_info,
            "cpu_baseline": cpu,
            "postprocess": postprocess,
        }
        print(json.dumps(out), flush=True)
    dev.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
