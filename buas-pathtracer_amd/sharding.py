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


def render_frame_sharded(render_shard, accum, rank, world, group=None, scratch=None, reduce=None):
    """render_shard(shard_index, shard_count, buf) ADDS this rank's tiles of one frame into
    `buf` (a torch tensor shaped like `accum`).  With world > 1 (or `reduce` set: the same path at
    one rank) the frame is rendered into `scratch` (zeroed here; allocated if None), sum-reduced
    into rank 0 and added to rank 0's `accum`; the other ranks' `accum` is left untouched.
    Returns the render_shard result."""
    if not (world > 1 if reduce is None else reduce):
        return render_shard(rank, world, accum)
    import torch.distributed as dist
    buf = scratch if scratch is not None else accum.new_zeros(accum.shape)
    buf.zero_()
    stats = render_shard(rank, world, buf)
    if buf.is_cuda and dist.get_backend(group) == "gloo":
        # gloo reduces host tensors: stage the frame through host memory (the CPU-side test path;
        # RCCL reduces the device buffer in place over xGMI)
        host = buf.cpu()
        dist.reduce(host, dst=0, group=group)
        if rank == 0:
            buf.copy_(host)
    else:
        dist.reduce(buf, dst=0, group=group)
    if rank == 0:
        accum.add_(buf)
    return stats
