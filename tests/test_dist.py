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


def _pipe_worker(rank, world, port, out_path, seeds):
    """Back-to-back frames through PipelinedExchange (the bench's N > 1 path):
    frame k (seed seeds[k]) renders into packed buffer k % 2 and is gathered
    into its own frame tensor."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dsgpuraytracing_amd.dist import PipelinedExchange
    from tests.oracle_helpers import Restatement, golden
    rs = Restatement()
    scene = golden("c1_default_64x64.scene.ptd")
    ntx = (W + 31) // 32
    pex = PipelinedExchange(tile_fifo(W, H), W, H, rank, world, torch.device("cpu"))
    frames = [torch.zeros((H, W, 3), dtype=torch.float32) for _ in seeds]
    for k, seed in enumerate(seeds):
        packed = pex.packed_for(k)
        assert packed.data_ptr() == pex.ex.bufs[k % 2].data_ptr()
        for i, (x, y, tw, th) in enumerate(pex.mine):
            idx = (y // 32) * ntx + x // 32
            img, _ = rs.render(scene, W, H, SPP, seed=seed, rng_mode=1, tile_begin=idx, tile_end=idx + 1)
            packed[i].view(32, 32, 3)[:th, :tw] = torch.from_numpy(img[y:y + th, x:x + tw])
        pex.exchange(k, frames[k], timed=True)
    pex.drain()
    if rank == 0:
        np.save(out_path, torch.stack(frames).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_pipelined_exchange_bit_identical_over_frames(tmp_path, restate, world):
    """Double-buffered packed tiles, frame after frame: every assembled frame
    equals the single-process render of its own seed bit for bit (a frame
    gathered from the wrong buffer would carry another seed's pixels)."""
    from tests.oracle_helpers import golden
    seeds = [3, 5, 8]
    out = str(tmp_path / "frames.npy")
    mp.spawn(_pipe_worker, args=(world, _free_port(), out, seeds), nprocs=world, join=True)
    got = np.load(out)
    for k, seed in enumerate(seeds):
        ref, _ = restate.render(golden("c1_default_64x64.scene.ptd"), W, H, SPP, seed=seed, rng_mode=1, threads=2)
        assert np.array_equal(got[k], ref), k
    assert not np.array_equal(got[0], got[1])


@pytest.mark.parametrize("deal", ["mod", "diag", "diag3", "auto"])
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


def _fail_worker(rank, world, port, out_dir, fail_rank):
    """Renders a few frames through render_sharded; `fail_rank`'s renderer
    raises in frame 1 (as a PtError from libptgpu.so would)."""
    import sys
    import time
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from dsgpuraytracing_amd.dist import RankFailure, init_from_env
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    init_from_env("gloo", timeout_s=20)
    frame = torch.zeros((H, W, 3), dtype=torch.float32)
    t0 = time.time()
    code = 0
    try:
        for k in range(3):
            def render(tiles, packed):
                if rank == fail_rank and k == 1:
                    raise RuntimeError("ptgpu error -2: hipErrorIllegalAddress (injected)")
                packed.fill_(float(rank + 1))
            render_sharded(render, frame, tile_fifo(W, H), rank, world)
        msg = "no failure"
    except RankFailure as e:
        msg = f"RankFailure frame {k}: {e} failed={e.failed}"
        code = 3
    with open(os.path.join(out_dir, f"rank{rank}.txt"), "w") as f:
        f.write(f"{time.time() - t0:.3f}\n{msg}\n")
    dist.destroy_process_group()
    sys.exit(code)


@pytest.mark.parametrize("world,fail_rank", [(2, 1), (3, 0)])
def test_failing_rank_stops_every_rank(tmp_path, world, fail_rank):
    """SURVEY §5 / VERDICT r2: a per-rank failure surfaces as an error from the
    exchange step on EVERY rank, promptly (not a process-group timeout), with
    the failing rank's message; every process exits non-zero."""
    import time
    ctx = mp.get_context("spawn")
    port = _free_port()
    ps = [ctx.Process(target=_fail_worker, args=(r, world, port, str(tmp_path), fail_rank)) for r in range(world)]
    t0 = time.time()
    for p in ps:
        p.start()
    for p in ps:
        p.join(60)
    assert all(not p.is_alive() for p in ps), "a rank is still blocked"
    assert [p.exitcode for p in ps] == [3] * world
    assert time.time() - t0 < 45
    for r in range(world):
        secs, msg = open(tmp_path / f"rank{r}.txt").read().splitlines()
        assert msg.startswith("RankFailure frame 1:"), msg
        assert f"rank {fail_rank}: RuntimeError: ptgpu error -2" in msg
        assert float(secs) < 15  # seconds, far below the 20 s group timeout


def _knob_worker(rank, world, port, out_dir, knob="PT_SAMPLE_GROUP", value="8"):
    import sys
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from dsgpuraytracing_amd.dist import RankFailure, check_value_knobs
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if rank == 1:
        os.environ[knob] = value
    else:
        os.environ.pop(knob, None)
    code = 0
    try:
        check_value_knobs({"group_spp": 4})
        msg = "ok"
    except RankFailure as e:
        msg = str(e)
        code = 3
    with open(os.path.join(out_dir, f"knob{rank}.txt"), "w") as f:
        f.write(msg)
    dist.destroy_process_group()
    sys.exit(code)


@pytest.mark.parametrize("knob,value", [("PT_SAMPLE_GROUP", "8"), ("PT_WAVES_PER_CU", "12"), ("PT_SAH_BINS", "64"),
                                        ("PT_SAH_CI", "1.5"), ("PT_SAH_LEAF", "2"), ("PT_NO_FOOTPRINT_CULL", "1")])
def test_value_knobs_must_agree(tmp_path, knob, value):
    """PT_SAMPLE_GROUP / PT_WAVES_PER_CU change each pixel's float summation
    order (the group size), the PT_SAH_* knobs the host SAH tree and so its
    tie-breaks, PT_NO_FOOTPRINT_CULL which pixels are traced: ranks that
    differ could break the bit-identity of the assembled frame, so the split
    refuses to start."""
    ctx = mp.get_context("spawn")
    port = _free_port()
    ps = [ctx.Process(target=_knob_worker, args=(r, 2, port, str(tmp_path), knob, value)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(60)
    assert [p.exitcode for p in ps] == [3, 3]
    for r in range(2):
        assert knob in open(tmp_path / f"knob{r}.txt").read()


def _packed16_worker(rank, world, port, out_path, deal, deal_block=0):
    """The strong split dealing 16x16 tiles (PT_FLAG_PACKED16 slots): each
    rank fills its packed slots from the frame (the restatement's whole-frame
    render, cheap at this size) and ONE gather + scatter assembles rank 0's."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dsgpuraytracing_amd.dist import TileExchange
    from tests.oracle_helpers import Restatement, golden
    img, _ = Restatement().render(golden("c1_default_64x64.scene.ptd"), W, H, SPP, rng_mode=1, threads=1)
    ex = TileExchange(tile_fifo(W, H, 16), W, H, rank, world, torch.device("cpu"), deal=deal, tile_size=16,
                      deal_block=deal_block)
    assert ex.slot == 16 and ex.packed.shape[1] == 256
    for i, (x, y, tw, th) in enumerate(ex.mine):
        ex.packed[i].view(16, 16, 3)[:th, :tw] = torch.from_numpy(img[y:y + th, x:x + tw])
    frame = torch.zeros((H, W, 3), dtype=torch.float32)
    ex.exchange(frame)
    if rank == 0:
        np.save(out_path, frame.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,deal,block", [(2, "diag3", 0), (3, "diag5", 0), (2, "auto", 32)])
def test_packed16_split_bit_identical(tmp_path, restate, world, deal, block):
    from tests.oracle_helpers import golden
    out = str(tmp_path / "frame16.npy")
    mp.spawn(_packed16_worker, args=(world, _free_port(), out, deal, block), nprocs=world, join=True)
    ref, _ = restate.render(golden("c1_default_64x64.scene.ptd"), W, H, SPP, rng_mode=1, threads=2)
    assert np.array_equal(np.load(out), ref)


@pytest.mark.parametrize("deal", ["diag", "diag3", "diag5"])
def test_shard_tiles_partition_16(deal):
    """16x16 tiles (bench.py --split-tile 16): a partition with equal counts
    up to one tile per row, columns / rows counted in 16-px tiles."""
    tiles = tile_fifo(1024, 1024, 16)
    for world in (2, 4, 8):
        shards = [shard_tiles(tiles, r, world, deal, 16) for r in range(world)]
        assert sorted(t for s in shards for t in s) == sorted(tiles)
        assert len({len(s) for s in shards}) == 1  # 64 x 64 tiles: exact
    from dsgpuraytracing_amd.dist import packed_index
    src, dst = packed_index([(0, 0, 16, 16), (16, 32, 8, 4)], 40, slot=16)
    k = int(np.nonzero(dst == 33 * 40 + 17)[0][0])
    assert src[k] == 256 + 1 * 16 + 1


def test_auto_deal_and_deal_blocks():
    """"auto" is diag3 at 8 or more ranks and diag below (the measured best:
    profiles/r6/ab_split_deal.txt); a deal by 32-px blocks keeps the four
    16x16 tiles of each block on one rank."""
    from dsgpuraytracing_amd.dist import tile_owner
    t32, t16 = tile_fifo(512, 256), tile_fifo(512, 256, 16)
    for world, k in ((2, "diag"), (4, "diag"), (8, "diag3"), (16, "diag3")):
        assert [tile_owner(t, i, world, "auto") for i, t in enumerate(t32)] == \
            [tile_owner(t, i, world, k) for i, t in enumerate(t32)]
    for world in (2, 8):
        own32 = {(t[0], t[1]): tile_owner(t, i, world, "diag3") for i, t in enumerate(t32)}
        for i, t in enumerate(t16):
            assert tile_owner(t, i, world, "diag3", 32) == own32[(t[0] // 32 * 32, t[1] // 32 * 32)]
        shards = [shard_tiles(t16, r, world, "diag3", 32) for r in range(world)]
        assert sorted(t for s in shards for t in s) == sorted(t16)
