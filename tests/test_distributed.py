"""World-size-2 gloo test of the multi-GPU decomposition on CPU: each rank
renders its interleaved tiles (t % 2 == rank) with the CPU oracle into a full
frame buffer, the buffers are sum-reduced with gloo (RCCL on the GPU box), and
the result must equal the single-rank frame up to float summation order."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

W, H = 128, 96


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    import conftest
    rt = conftest._import_package()
    import oracle_binding as ob
    from buas_pathtracer_amd.sharding import render_frame_sharded, owned_tiles
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scene, cam, st, fc, post = rt.load_preset("c1", W, H)
    st.samples_per_pixel = 4
    accum = torch.zeros((H, W, 4), dtype=torch.float32)

    def render_shard(shard_index, shard_count, buf):
        a = buf.numpy()
        _, stats = ob.render(scene.desc(), cam, st, fc, W, H, rng_mode=0, threads=2, accum=a,
                             shard_index=shard_index, shard_count=shard_count)
        return stats.samples

    samples = render_frame_sharded(render_shard, accum, rank, world)
    n = torch.tensor([samples], dtype=torch.float64)
    dist.all_reduce(n)
    if rank == 0:
        np.save(out_path, accum.numpy())
        with open(out_path + ".n", "w") as f:
            f.write(str(int(n.item())))
    assert len(owned_tiles(W, H, 64, 64, rank, world)) >= 1
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_matches_single(rt, tmp_path):
    import oracle_binding as ob
    out = str(tmp_path / "frame.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    reduced = np.load(out)
    scene, cam, st, fc, post = rt.load_preset("c1", W, H)
    st.samples_per_pixel = 4
    full, stats = ob.render(scene.desc(), cam, st, fc, W, H, rng_mode=0, threads=2)
    assert int(open(out + ".n").read()) == stats.samples == W * H * 4
    err = np.linalg.norm((reduced - full).astype(np.float64)) / np.linalg.norm(full.astype(np.float64))
    assert err <= 1e-6


def test_owned_tiles_partition(rt):
    from buas_pathtracer_amd.sharding import owned_tiles
    for world in (1, 2, 3, 8):
        tiles = sorted(t for r in range(world) for t in owned_tiles(1920, 1080, 64, 64, r, world))
        assert tiles == list(range(30 * 17))
