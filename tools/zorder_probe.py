"""Diagnostic: one C5 frame through the library, printing whether the launch
took the Z-ordered tile list (pt_stats.tile_zorder) and the render-tree size
the rule reads (round 6 session an)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dsgpuraytracing_amd.pathtracer import Device, Scene, tile_fifo  # noqa: E402

wl = bench.WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "c5"]
dae, envmap, cam = bench.workload_scene(wl)
sc = Scene.from_dae(dae, wl["w"], wl["h"], cam_info=cam, envmap=envmap)
torch.cuda.set_device(0)
dev = Device(0)
dev.upload_scene(sc)
dev.set_camera(sc.camera)
dev.set_params(wl["w"], wl["h"], wl["spp"], 4, 1, 1)
frame = torch.zeros((wl["h"] * wl["w"] * 3,), dtype=torch.float32, device="cuda:0")
tiles = np.asarray(tile_fifo(wl["w"], wl["h"]), np.int32)
for _ in range(2):
    t = time.perf_counter()
    dev.render_tiles_device(tiles, frame.data_ptr())
    torch.cuda.synchronize()
    st = dev.stats()
    print(wl["w"], wl["h"], "zorder", st["tile_zorder"], "ms", round((time.perf_counter() - t) * 1e3, 2),
          {k: st[k] for k in st if "node" in k and not isinstance(st[k], list)}, flush=True)
dev.close()
