"""GPU linear-BVH build (pt_upload_scene_lbvh, csrc/lbvh.hip) — the reference's
PARALLEL_BUILD_BVH path (cuda_src/setup.cu:478-686, kernel.cu:358-493).

The reference's CUDA builder cannot run here (no CUDA), so parity is anchored
on what a BVH must not change: nearest hits, occlusion answers and rendered
images, against the reference's own ray-query answers (BVHAccel::intersect,
tests/golden/c1_rays_ref.ptd) and against renders through the reference's
host-built BVH."""
import os

import numpy as np
import pytest

from dsgpuraytracing_amd import native, ptdump, scenes
from dsgpuraytracing_amd.pathtracer import Device, PathTracer, Scene
from tests.oracle_helpers import golden

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _render(sc, w, h, spp, seed, gpu_bvh, **kw):
    pt = PathTracer(ns_aa=spp, max_ray_depth=4, ns_area_light=1, seed=seed, gpu_bvh=gpu_bvh, **kw)
    pt.set_frame_size(w, h)
    pt.set_camera(sc.camera)
    pt.set_scene(sc)
    pt.start_raytracing(stats=True)
    return pt.sampleBuffer.copy(), pt.last_stats


def _close(a, b):
    diff = np.abs(a - b).max(axis=2)
    return (diff <= 1e-3 * np.maximum(1.0, np.abs(b).max(axis=2))).mean()


def test_lbvh_ray_queries_vs_reference_kat():
    rays = ptdump.read(golden("c1_rays.ptd"))
    ref = ptdump.read(golden("c1_rays_ref.ptd"))
    dev = Device(0)
    dev.upload_scene(Scene.from_dump(golden("c1_default_64x64.scene.ptd")), gpu_bvh=True)
    hit, t, prim, anyh = dev.intersect(rays["ray_o"], rays["ray_d"], rays["ray_maxt"])
    assert (hit == ref["hit"]).mean() >= 0.995
    both = (hit == 1) & (ref["hit"] == 1)
    assert (prim[both] == ref["prim"][both]).mean() >= 0.99   # uploaded-order ids (prim_map)
    assert (anyh == ref["any"]).mean() >= 0.995


@pytest.mark.parametrize("name", ["c1_default_64x64", "CBspheres_64x64", "c1env_64x64"])
def test_lbvh_render_matches_reference_bvh(name):
    sc = Scene.from_dump(golden(f"{name}.scene.ptd"))
    a, _ = _render(sc, 64, 64, 4, 3, gpu_bvh=False)
    b, st = _render(sc, 64, 64, 4, 3, gpu_bvh=True)
    assert _close(b, a) >= 0.999
    assert st["bvh_nodes"] >= 1


def test_lbvh_bunny_matches_reference_bvh():
    """28,576-triangle bunny: the GPU-built tree gives the same image."""
    sc = Scene.from_dae(os.path.join(ROOT, "assets", "CBbunny.dae"), 96, 96)
    a, sa = _render(sc, 96, 96, 2, 5, gpu_bvh=False)
    b, sb = _render(sc, 96, 96, 2, 5, gpu_bvh=True)
    assert _close(b, a) >= 0.999
    assert abs(b.mean() - a.mean()) <= 1e-3 * a.mean()
    assert sb["bvh_nodes"] > 1000 and sb["bvh_stack"] >= 3


def test_pathtracer_envmap_argument_equals_scene_envmap():
    """PathTracer(envmap=...) appends the EnvironmentLight like the reference
    constructor does; the result equals the scene that already carries it."""
    base = Scene.from_dump(golden("c1_default_64x64.scene.ptd"))
    with_env = Scene.from_dump(golden("c1env_64x64.scene.ptd"))
    a, _ = _render(with_env, 64, 64, 2, 7, gpu_bvh=False)
    b, _ = _render(base, 64, 64, 2, 7, gpu_bvh=False, envmap=golden("env_sky_64x32.exr"))
    assert np.array_equal(a, b)


@pytest.mark.parametrize("passes", ["0", "1", "2", "3"])
def test_lbvh_treelet_restructuring_keeps_nearest_hits(monkeypatch, passes):
    """The treelet-restructured GPU tree (Karras & Aila 2013; PT_LBVH_PASSES
    passes, 0 = the Karras tree with SAH leaf collapse) on the 114k-triangle
    C3 proxy: every ray query answers as over the host SAH tree (nearest hit,
    primitive in the caller's order, distance, occlusion), a frame renders
    near-exactly, and the restructured tree is not worse by the kernel's own
    traversal counters."""
    monkeypatch.setenv("PT_LBVH_PASSES", passes)
    sc = Scene.from_dae(scenes.proxy_path(1), 128, 128)
    rng = np.random.default_rng(17)
    m = 20000
    d = sc.arrays.d
    g = np.asarray(d["prim_geom"]).reshape(-1, 9)
    lo, hi = g[:, :3].min(0), g[:, :3].max(0)
    o = lo + rng.uniform(-0.2, 1.2, (m, 3)) * (hi - lo)
    pick = rng.integers(0, len(g), m)  # aim at triangle interiors (vertices and edges are shared: ties)
    bc = rng.dirichlet([2.0, 2.0, 2.0], m)
    tgt = (g[pick].reshape(m, 3, 3) * bc[:, :, None]).sum(1)
    dr = tgt - o
    dr /= np.linalg.norm(dr, axis=1, keepdims=True)
    maxt = rng.uniform(0.1, 3.0, m)
    res = []
    for gpu in (False, True):
        if gpu:
            monkeypatch.delenv("PT_BVH_BUILD", raising=False)
        else:  # the host binned-SAH tree
            monkeypatch.setenv("PT_BVH_BUILD", "sah")
        dev = Device(0)
        dev.upload_scene(sc, gpu_bvh=gpu)
        res.append(dev.intersect(o, dr, maxt))
        dev.close()
    (h0, t0, p0, a0), (h1, t1, p1, a1) = res
    assert h0.mean() > 0.5
    assert (h0 == h1).mean() >= 0.9995 and (a0 == a1).mean() >= 0.9995
    both = (h0 == 1) & (h1 == 1)
    # the same nearest primitive, or a tie at the same distance (coplanar or
    # shared-edge triangles: which one a tree reports first is the tree's)
    assert ((p0[both] == p1[both]) | (t0[both] == t1[both])).mean() >= 0.9995
    assert np.allclose(t0[both], t1[both], rtol=1e-6, atol=0)
    monkeypatch.setenv("PT_BVH_BUILD", "sah")
    a, sa = _render(sc, 128, 128, 4, 9, gpu_bvh=False)
    monkeypatch.delenv("PT_BVH_BUILD", raising=False)
    b, sb = _render(sc, 128, 128, 4, 9, gpu_bvh=True)
    assert _close(b, a) >= 0.999
    print(f"passes {passes}: BVH4 nodes {sb['bvh_nodes']} (host {sa['bvh_nodes']}), node visits {sb['node_visits']} "
          f"(host {sa['node_visits']}), tri tests {sb['tri_tests']} (host {sa['tri_tests']}), "
          f"wave steps {sb['wave_trav_steps']} (host {sa['wave_trav_steps']})")
