"""Upload (scene conversion + render-tree build) timing on the GPU box: the C3
and C5 scenes uploaded twice each (the second, warm, time is printed), for the
render tree selected by the environment (PT_BVH_BUILD, PT_LBVH_PASSES).
Usage: python tools/upload_timing.py [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dsgpuraytracing_amd import scenes  # noqa: E402
from dsgpuraytracing_amd.pathtracer import Device, Scene  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    c3 = Scene.from_dae(scenes.proxy_path(1), 1024, 1024)
    c5 = Scene.from_dae(scenes.c5_path(2), 1920, 1080, envmap=scenes.c5_envmap_path())
    d = Device(0)
    out = {}
    for name, sc in (("c3", c3), ("c5", c5)):
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            d.upload_scene(sc)
            ts.append(time.perf_counter() - t)
        out[name] = round(min(ts[1:] or ts) * 1e3, 1)
    print(os.environ.get("PT_BVH_BUILD", "gpu"), os.environ.get("PT_LBVH_PASSES", "default"), out, flush=True)


if __name__ == "__main__":
    main()
