"""RCCL (torch.distributed "nccl") on the box, in the exact call pattern of
bench.py's multi-GPU path: every collective the N-GPU run issues (gather of
packed tiles onto rank 0, sum-reduce of passes, MAX all-reduce of the timed
region, all-gather of per-rank timings, barriers), on CUDA tensors with a
dedicated current stream, after a render queued on that stream.  One rank
(the box has one GPU; the 8-rank run is the driver's): this pins the RCCL
runtime and the stream ordering, not the link bandwidth.  The multi-rank
semantics of the same calls are covered with gloo in tests/test_dist.py."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_collectives_after_device_render():
    import torch
    import torch.distributed as dist

    from dsgpuraytracing_amd.dist import TileExchange
    from dsgpuraytracing_amd.pathtracer import Device, Scene, tile_fifo
    from tests.oracle_helpers import golden

    torch.cuda.set_device(0)
    stream = torch.cuda.Stream(device=0)
    torch.cuda.set_stream(stream)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        w = h = 64
        sc = Scene.from_dump(golden("c1_default_64x64.scene.ptd"))
        dev = Device(0)
        dev.upload_scene(sc)
        dev.set_camera(sc.camera)
        dev.set_params(w, h, 2, 4, 1, 1)
        tiles = tile_fifo(w, h)
        ex = TileExchange(tiles, w, h, 0, 1, torch.device("cuda", 0))
        frame = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda:0")
        mine = np.asarray(ex.mine, dtype=np.int32).reshape(-1, 4)
        dev.render_tiles_device(mine, ex.packed.data_ptr(), stream.cuda_stream, packed=True)
        # the packed-tile gather exactly as TileExchange issues it for N > 1
        gl = list(ex.recv.unbind(0))
        dist.gather(ex.packed, gather_list=gl, dst=0)
        ex.scatter(frame)
        ref = torch.zeros_like(frame)
        dev.render_tiles_device(np.asarray(tiles, np.int32).reshape(-1, 4), ref.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(frame, ref) and float(ref.mean()) > 0
        # weak-scaling pass reduction, timing MAX, per-rank table, barrier
        red = ref.clone()
        dist.reduce(red, dst=0)
        t = torch.tensor([1.5], dtype=torch.float64, device="cuda:0")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        allr = [torch.zeros(4, dtype=torch.float64, device="cuda:0")]
        dist.all_gather(allr, torch.arange(4, dtype=torch.float64, device="cuda:0"))
        dist.barrier()
        torch.cuda.synchronize()
        assert torch.equal(red, ref) and float(t.item()) == 1.5
        assert allr[0].tolist() == [0.0, 1.0, 2.0, 3.0]
    finally:
        dist.destroy_process_group()
        torch.cuda.set_stream(torch.cuda.default_stream(0))


@pytest.mark.parametrize("side", [False, True])
def test_pipelined_exchange_on_device_keeps_every_frame(side):
    """bench.py's N > 1 default in its exact stream pattern on the box: frames
    rendered back to back (on the library's render-slot streams) into
    double-buffered packed tiles, each frame's RCCL gather + scatter queued
    behind its resolve on the current stream (side=False, the default) or on
    a side stream behind an event (side=True) while the next frame renders.  Every frame (its own seed) must equal its direct whole-
    frame render bit for bit: a gather reading a buffer the next-but-one
    render already overwrote, or a scatter racing the gather, would not."""
    import torch
    import torch.distributed as dist

    from dsgpuraytracing_amd.dist import PipelinedExchange
    from dsgpuraytracing_amd.pathtracer import Device, Scene, tile_fifo
    from tests.oracle_helpers import golden

    torch.cuda.set_device(0)
    stream = torch.cuda.Stream(device=0)
    torch.cuda.set_stream(stream)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        w = h = 128
        spp = 8
        sc = Scene.from_dump(golden("c1_default_128x128.scene.ptd"))
        dev = Device(0)
        dev.upload_scene(sc)
        dev.set_camera(sc.camera)
        tiles = tile_fifo(w, h)
        pex = PipelinedExchange(tiles, w, h, 0, 1, torch.device("cuda", 0), side=side)
        mine = np.asarray(pex.mine, dtype=np.int32).reshape(-1, 4)
        seeds = [11, 12, 13, 14, 15]
        frames = [torch.zeros((h, w, 3), dtype=torch.float32, device="cuda:0") for _ in seeds]
        for k, seed in enumerate(seeds):  # nothing waits on the host between frames
            dev.set_params(w, h, spp, 4, 1, seed)
            buf = pex.packed_for(k)
            dev.render_tiles_device(mine, buf.data_ptr(), stream.cuda_stream, packed=True, out_floats=buf.numel())
            pex.exchange(k, frames[k], timed=True)
        pex.drain()
        torch.cuda.synchronize()
        assert pex.exchange_ms() > 0
        whole = np.asarray(tiles, np.int32).reshape(-1, 4)
        for k, seed in enumerate(seeds):
            ref = torch.zeros_like(frames[k])
            dev.set_params(w, h, spp, 4, 1, seed)
            dev.render_tiles_device(whole, ref.data_ptr(), stream.cuda_stream)
            torch.cuda.synchronize()
            assert torch.equal(frames[k], ref), k
            assert float(ref.mean()) > 0
        assert not torch.equal(frames[0], frames[1])
        dev.close()
    finally:
        dist.destroy_process_group()
        torch.cuda.set_stream(torch.cuda.default_stream(0))
