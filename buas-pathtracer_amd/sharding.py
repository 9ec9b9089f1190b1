"""Multi-GPU decomposition of a frame.

Tile t of the frame is rendered by rank t % world (interleaved for load balance, the
reference's 64x64 tiles).  Every rank renders its share of the frame into a full-frame
float4 buffer that starts the frame at zero (only its tiles' splats are non-zero), one sum
reduction over the ranks (RCCL over xGMI on MI355X, gloo in the CPU tests) combines the
shares in rank 0, and rank 0 adds the frame to its accumulation buffer.  Samples are keyed by
(frame, tile, pixel, sample), so the result does not depend on the number of ranks beyond
float summation order.

Progressive accumulation (frame_count > 0, RT/raytracer.cpp:720-724) is therefore safe: the
accumulation buffer of a rank other than 0 is never read or changed, and rank 0's earlier
frames are reduced with nobody else's.
"""


def owned_tiles(w, h, tile_w, tile_h, rank, world):
    """Tile indices rank `rank` renders, in the reference's processing order (descending)."""
    tcx = (w + tile_w - 1) // tile_w
    tcy = (h + tile_h - 1) // tile_h
    return [t for t in range(tcx * tcy - 1, -1, -1) if t % world == rank]


def render_frame_sharded(render_shard, accum, rank, world, group=None, scratch=None, reduce=None, timing=None):
    """render_shard(shard_index, shard_count, buf) ADDS this rank's tiles of one frame into
    `buf` (a torch tensor shaped like `accum`).  With world > 1 (or `reduce` set: the same path at
    one rank) the frame is rendered into `scratch` (zeroed here; allocated if None), sum-reduced
    into rank 0 and added to rank 0's `accum`; the other ranks' `accum` is left untouched.
    Returns the render_shard result.

    timing (a dict, optional) collects per call: "render_s" (host wall time of render_shard, which
    returns once the frame is done on the device) and, on the reduce path, "reduce_s" (host wall
    time of a host-tensor reduce) or "reduce_events" (a pair of CUDA events around a device-tensor
    reduce on the current stream; RCCL's stream is joined to it, read them after a synchronize)."""
    import time
    if not (world > 1 if reduce is None else reduce):
        t0 = time.perf_counter()
        stats = render_shard(rank, world, accum)
        if timing is not None:
            timing.setdefault("render_s", []).append(time.perf_counter() - t0)
        return stats
    import torch
    import torch.distributed as dist
    buf = scratch if scratch is not None else accum.new_zeros(accum.shape)
    buf.zero_()
    t0 = time.perf_counter()
    stats = render_shard(rank, world, buf)
    t1 = time.perf_counter()
    if timing is not None:
        timing.setdefault("render_s", []).append(t1 - t0)
    if buf.is_cuda and dist.get_backend(group) == "gloo":
        # gloo reduces host tensors: stage the frame through host memory (the CPU-side test path;
        # RCCL reduces the device buffer in place over xGMI)
        host = buf.cpu()
        dist.reduce(host, dst=0, group=group)
        if rank == 0:
            buf.copy_(host)
        if timing is not None:
            timing.setdefault("reduce_s", []).append(time.perf_counter() - t1)
    elif buf.is_cuda and timing is not None:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        dist.reduce(buf, dst=0, group=group)
        ev[1].record()
        timing.setdefault("reduce_events", []).append(ev)
    else:
        dist.reduce(buf, dst=0, group=group)
        if timing is not None:
            timing.setdefault("reduce_s", []).append(time.perf_counter() - t1)
    if rank == 0:
        accum.add_(buf)
    return stats


def timing_summary(timing):
    """Per-call milliseconds from a render_frame_sharded timing dict (call after a synchronize):
    {"render_ms": [...], "reduce_ms": [...]} (reduce_ms empty without a reduce)."""
    out = {"render_ms": [1e3 * t for t in timing.get("render_s", [])],
           "reduce_ms": [1e3 * t for t in timing.get("reduce_s", [])]}
    out["reduce_ms"] += [a.elapsed_time(b) for a, b in timing.get("reduce_events", [])]
    return out
