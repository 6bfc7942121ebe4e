"""Diagnostic: trace one pixel's paths on the GPU (printf from the DBG kernel
variant) for a golden C1 scene.  Usage:
  PT_DEBUG_PIXEL=x,y python tools/debug_pixel.py <scene> W H spp depth l seed"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.test_gpu_render import gpu_render  # noqa: E402

scene, w, h, spp, m, l, seed = sys.argv[1], *map(int, sys.argv[2:8])
img, _ = gpu_render(scene, w, h, spp, m, l, seed)
x, y = map(int, os.environ["PT_DEBUG_PIXEL"].split(","))
print("pixel value", img[y, x])
