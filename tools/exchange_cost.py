"""On-device cost of the strong split's exchange on ONE GPU (the xGMI link
time of the gather itself needs the 8-GPU node): for the C3 frame dealt over
N = 2 / 4 / 8 ranks, the bytes each rank sends, rank 0's scatter of the N
gathered packed buffers into the frame (HIP events, index_select +
index_copy), and the HOST time to issue one frame of one rank's share -- the
render call plus the pipelined exchange's calls, nothing synchronised -- next
to that share's device time per frame: a split whose host issue time exceeds
its render time is host-bound.  Also the gather's lower bound at one xGMI
link (MI355X_MICROARCH.md: 7 links x ~153 GB/s per GPU; every sender uses its
own link into rank 0).  Usage: python tools/exchange_cost.py"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from dsgpuraytracing_amd import scenes  # noqa: E402
from dsgpuraytracing_amd.dist import PipelinedExchange, TileExchange, shard_tiles  # noqa: E402
from dsgpuraytracing_amd.pathtracer import Device, Scene, tile_fifo  # noqa: E402

W, H, SPP = 1024, 1024, 64
LINK_GBS = 153.0


def main():
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream(device=0)
    torch.cuda.set_stream(stream)
    sc = Scene.from_dae(scenes.proxy_path(1), W, H)
    dev = Device(0)
    dev.upload_scene(sc)
    dev.set_camera(sc.camera)
    dev.set_params(W, H, SPP, 4, 1, 1)
    tiles = tile_fifo(W, H)
    frame = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda:0")
    for n in (2, 4, 8):
        ex = TileExchange(tiles, W, H, 0, n, frame.device)  # rank 0's view: recv holds N packed buffers
        ex.recv.uniform_()
        for _ in range(3):
            ex.scatter(frame)
        ev = []
        for _ in range(20):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            ex.scatter(frame)
            b.record()
            ev.append((a, b))
        torch.cuda.synchronize()
        scatter_ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
        send = int(ex.packed.numel() * 4)
        # host issue time of one rank's frame (render + pipelined exchange), rank 0's share
        share = shard_tiles([(x, y, min(w, W - x), min(h, H - y)) for (x, y, w, h) in tiles], 0, n, "diag")
        pex = PipelinedExchange(share, W, H, 0, 1, frame.device)
        mine = np.asarray(pex.mine, np.int32).reshape(-1, 4)

        def one(k):
            buf = pex.packed_for(k)
            dev.render_tiles_device(mine, buf.data_ptr(), stream.cuda_stream, packed=True, out_floats=buf.numel())
            pex.exchange(k, frame)

        for k in range(4):
            one(k)
        torch.cuda.synchronize()
        frames = 30
        t0 = time.perf_counter()
        for k in range(4, 4 + frames):
            one(k)
        t_issue = (time.perf_counter() - t0) / frames
        pex.drain()
        torch.cuda.synchronize()
        t_all = (time.perf_counter() - t0) / frames
        k_ms, _ = dev.launch_times(frames)
        print(json.dumps({"n": n, "send_bytes_per_rank": send, "gather_link_bound_us": round(send / (LINK_GBS * 1e3), 1),
                          "rank0_scatter_ms": round(scatter_ms, 4), "host_issue_ms_per_frame": round(t_issue * 1e3, 4),
                          "frame_ms_share_pipelined": round(t_all * 1e3, 4),
                          "render_event_ms_share": round(float(np.mean(k_ms)), 4), "share_tiles": len(share)}),
              flush=True)
    dev.close()


if __name__ == "__main__":
    main()
