"""Bit-identity check between library builds: renders a fixed set of frames
with the library PT_LIB names (or the in-tree one) and prints one sha256 per
frame of the HDR sampleBuffer.  Run once per build on the GPU box and diff
the lines.  Usage: PT_LIB=_variants/x.so python tools/img_hash.py"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dsgpuraytracing_amd import scenes  # noqa: E402
from dsgpuraytracing_amd.pathtracer import Device, Scene, tile_fifo  # noqa: E402

A = os.path.join(ROOT, "assets")
CASES = [  # name, dae, envmap, cam, w, h, spp, depth, nsl
    ("c3_128", scenes.proxy_path(1), None, None, 256, 256, 16, 4, 1),
    ("c5_256", scenes.c5_path(2), scenes.c5_envmap_path(), None, 320, 180, 16, 4, 1),
    ("spheres_l3", os.path.join(A, "CBspheres.dae"), None, None, 128, 128, 8, 5, 3),
    ("point", os.path.join(A, "CBspheres_lambertian_pointlight.dae"), None, None, 128, 128, 8, 4, 2),
    ("dir", os.path.join(A, "CBspheres_lambertian_dirlight.dae"), None, None, 128, 128, 8, 4, 1),
    ("hemi", os.path.join(A, "CBspheres_lambertian_ambientlight.dae"), None, None, 128, 128, 8, 4, 2),
    ("refr", os.path.join(A, "CBspheres_refraction.dae"), None, None, 128, 128, 8, 6, 1),
]
for name, dae, env, cam, w, h, spp, depth, nsl in CASES:
    sc = Scene.from_dae(dae, w, h, cam_info=cam, envmap=env)
    dev = Device(0)
    dev.upload_scene(sc)
    dev.set_camera(sc.camera)
    dev.set_params(w, h, spp, depth, nsl, 7)
    out = np.zeros((h, w, 3), np.float32)
    dev.render_tiles(tile_fifo(w, h), out)
    dev.close()
    print(name, hashlib.sha256(out.tobytes()).hexdigest()[:16], f"{float(out.mean()):.6f}", flush=True)
    if os.environ.get("IMG_SAVE"):  # directory for the frames (offline diffs between builds)
        os.makedirs(os.environ["IMG_SAVE"], exist_ok=True)
        np.save(os.path.join(os.environ["IMG_SAVE"], name + ".npy"), out)
