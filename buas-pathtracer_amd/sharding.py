"""Multi-GPU decomposition of a frame.

Tile t of the frame is rendered by rank t % world (interleaved for load
balance, the reference's 64x64 tiles), every rank accumulates into a full-frame
float4 buffer in which only its tiles' splats are non-zero, and one sum
reduction over the ranks (RCCL over xGMI on MI355X, gloo in the CPU tests)
produces the frame.  Samples are keyed by (frame, tile, pixel, sample), so the
result does not depend on the number of ranks beyond float summation order.
"""


def owned_tiles(w, h, tile_w, tile_h, rank, world):
    """Tile indices rank `rank` renders, in the reference's processing order (descending)."""
    tcx = (w + tile_w - 1) // tile_w
    tcy = (h + tile_h - 1) // tile_h
    return [t for t in range(tcx * tcy - 1, -1, -1) if t % world == rank]


def render_frame_sharded(render_shard, accum, rank, world, group=None):
    """render_shard(shard_index, shard_count, accum) adds this rank's tiles into
    `accum` (a torch tensor); the frame is then sum-reduced into rank 0's buffer.
    Returns the render_shard result (per-rank stats)."""
    import torch.distributed as dist
    stats = render_shard(rank, world, accum)
    if world > 1:
        dist.reduce(accum, dst=0, group=group)
    return stats
