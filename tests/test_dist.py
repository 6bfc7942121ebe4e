"""Multi-process tile sharding + packed-tile gather (gloo, CPU): the assembled
image must be bit-identical to a single-process render for any world size.
The per-rank renderer here is the oracle restatement in counter-RNG mode (the
HIP path uses the same RNG keys; tests/test_gpu_render.py checks HIP tiles
against whole frames on the GPU)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dsgpuraytracing_amd.dist import render_sharded, shard_tiles
from dsgpuraytracing_amd.pathtracer import tile_fifo

W, H = 96, 80  # ragged last tile row
SPP = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests.oracle_helpers import Restatement, golden
    rs = Restatement()
    scene = golden("c1_default_64x64.scene.ptd")
    frame = torch.zeros((H, W, 3), dtype=torch.float32)
    ntx = (W + 31) // 32

    def render(tiles, packed):  # the PT_FLAG_PACKED layout: tile i at packed[i], 32 px per row
        for i, (x, y, tw, th) in enumerate(tiles):
            idx = (y // 32) * ntx + x // 32
            img, _ = rs.render(scene, W, H, SPP, rng_mode=1, tile_begin=idx, tile_end=idx + 1)
            slot = packed[i].view(32, 32, 3)
            slot[:th, :tw] = torch.from_numpy(img[y:y + th, x:x + tw])

    render_sharded(render, frame, tile_fifo(W, H), rank, world)
    if rank == 0:
        np.save(out_path, frame.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_render_bit_identical(tmp_path, restate, world):
    from tests.oracle_helpers import golden
    out = str(tmp_path / "frame.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = np.load(out)
    ref, _ = restate.render(golden("c1_default_64x64.scene.ptd"), W, H, SPP, rng_mode=1, threads=2)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("deal", ["mod", "diag", "diag3"])
def test_shard_tiles_partition(deal):
    tiles = tile_fifo(1920, 1080)
    for world in (1, 2, 4, 8):
        shards = [shard_tiles(tiles, r, world, deal) for r in range(world)]
        flat = sorted(t for s in shards for t in s)
        assert flat == sorted(tiles)
        sizes = [len(s) for s in shards]
        assert max(sizes) - min(sizes) <= (1 if deal == "mod" else 34)  # diag: <= one tile per row
    with pytest.raises(ValueError):
        shard_tiles(tiles, 2, 2)


def test_packed_index_layout():
    from dsgpuraytracing_amd.dist import packed_index
    tiles = [(0, 0, 32, 32), (32, 64, 8, 16)]
    src, dst = packed_index(tiles, 40)
    assert len(src) == 32 * 32 + 8 * 16
    # tile 1's pixel (33, 65) -> slot 1, local (1, 1)
    k = int(np.nonzero(dst == 65 * 40 + 33)[0][0])
    assert src[k] == 1024 + 1 * 32 + 1
    assert len(set(dst.tolist())) == len(dst)
