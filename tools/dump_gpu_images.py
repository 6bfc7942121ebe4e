"""Diagnostic: render the near-exact test cases on the GPU and save the images
(gpurun_out/gpu_<case>.npy) for offline comparison with the restatement."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.test_gpu_render import gpu_render  # noqa: E402

os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
for scene, w, h, spp, m, l, seed in [("c1_default_64x64", 64, 64, 4, 4, 1, 1), ("c1_sphcam_96x64", 96, 64, 3, 4, 2, 7),
                                     ("c1_default_128x128", 128, 128, 16, 4, 1, 3)]:
    img, st = gpu_render(scene, w, h, spp, m, l, seed, stats=True)
    np.save(os.path.join(ROOT, "gpurun_out", f"gpu_{scene}_s{spp}_seed{seed}.npy"), img)
    print(scene, st)
