"""The render tree pt_upload_scene traverses (csrc/render_tree.cpp,
pt_host_build_render_tree), checked on the CPU: a valid BVH
over exactly the scene's primitives (ranges partition their parent's, boxes
contain their children and primitives, leaves of <= 4 primitives), the same
tree for any host thread count, and the error paths.  The GPU side (hits and
frames over this tree equal those over the reference's tree) is in
tests/test_gpu_render.py."""
import ctypes
import os

import numpy as np
import pytest

from dsgpuraytracing_amd import native, ptdump, scenes
from dsgpuraytracing_amd.pathtracer import Scene
from tests.oracle_helpers import golden

NODE = np.dtype([("bb", "<f8", 6), ("info", "<i8", 4)])  # pt_bvh_node: box, start, range, left, right


def build(sc, threads=None, monkeypatch=None):
    if threads is not None:
        monkeypatch.setenv("PT_BUILD_THREADS", str(threads))
    n = sc.arrays.scene.n_prims
    nodes = np.zeros(max(1, 2 * n - 1), NODE)
    perm = np.zeros(n, np.int64)
    nn = ctypes.c_int64(0)
    rc = native.lib().pt_host_build_render_tree(ctypes.byref(sc.arrays.scene), nodes.ctypes.data, ctypes.byref(nn),
                                                perm.ctypes.data)
    assert rc == 0, native.lib().pt_last_error()
    return nodes[:nn.value], perm


def prim_boxes(sc):
    a = sc.arrays
    g = a.prim_geom.reshape(-1, 9)
    tri = a.prim_type == 1
    lo = np.where(tri[:, None], np.minimum(np.minimum(g[:, 0:3], g[:, 3:6]), g[:, 6:9]),
                  g[:, 0:3] - np.abs(g[:, 3:4]))
    hi = np.where(tri[:, None], np.maximum(np.maximum(g[:, 0:3], g[:, 3:6]), g[:, 6:9]),
                  g[:, 0:3] + np.abs(g[:, 3:4]))
    return lo, hi


def validate(sc, nodes, perm, max_leaf=4):
    n = sc.arrays.scene.n_prims
    assert np.array_equal(np.sort(perm), np.arange(n))
    plo, phi = prim_boxes(sc)
    seen = np.zeros(n, np.int64)
    stack, leaves = [0], 0
    start, rng, left, right = (nodes["info"][:, k] for k in range(4))
    while stack:
        i = stack.pop()
        lo, hi = nodes["bb"][i, :3], nodes["bb"][i, 3:]
        s, r = start[i], rng[i]
        idx = perm[s:s + r]
        assert np.all(plo[idx] >= lo) and np.all(phi[idx] <= hi)
        if left[i] < 0:
            assert right[i] < 0 and 1 <= r <= max_leaf
            seen[idx] += 1
            leaves += 1
            continue
        l, rr = left[i], right[i]
        assert start[l] == s and start[rr] == s + rng[l] and rng[l] + rng[rr] == r and rng[l] > 0 and rng[rr] > 0
        for c in (l, rr):
            assert np.all(nodes["bb"][c, :3] >= lo) and np.all(nodes["bb"][c, 3:] <= hi)
            stack.append(c)
    assert np.all(seen == 1)
    return leaves


def canonical(nodes):
    out, stack = [], [0]
    while stack:
        i = stack.pop()
        out.append((tuple(nodes["bb"][i]), int(nodes["info"][i, 0]), int(nodes["info"][i, 1])))
        if nodes["info"][i, 2] >= 0:
            stack += [int(nodes["info"][i, 3]), int(nodes["info"][i, 2])]
    return out


@pytest.mark.parametrize("name", ["c1_default_64x64", "CBspheres_64x64", "c1env_64x64"])
def test_render_tree_valid_small_scenes(name):
    sc = Scene.from_dump(golden(f"{name}.scene.ptd"))
    nodes, perm = build(sc)
    validate(sc, nodes, perm)


def test_render_tree_c3_proxy_valid_and_thread_independent(monkeypatch):
    sc = Scene.from_dae(scenes.proxy_path(1), 64, 64)
    trees = [build(sc, t, monkeypatch) for t in (1, 3, 8)]
    leaves = validate(sc, *trees[0])
    assert leaves > sc.arrays.scene.n_prims // 4
    for nodes, perm in trees[1:]:
        assert np.array_equal(perm, trees[0][1])
        assert canonical(nodes) == canonical(trees[0][0])


def test_render_tree_coincident_centroids():
    d = dict(ptdump.read(golden("c1_default_64x64.scene.ptd")))
    tri = int(np.flatnonzero(d["prim_type"] == 1)[0])
    for key in ("prim_geom", "prim_norm"):
        a = d[key].reshape(-1, 9)
        d[key] = np.concatenate([a, np.repeat(a[tri:tri + 1], 40, 0)]).reshape(-1)
    for key in ("prim_type", "prim_bsdf", "prim_orig"):
        d[key] = np.concatenate([d[key], np.repeat(d[key][tri:tri + 1], 40)])
    sc = Scene(native.SceneArrays(d))
    nodes, perm = build(sc)
    validate(sc, nodes, perm)


def test_render_tree_error_paths():
    lib = native.lib()
    sc = Scene.from_dump(golden("c1_default_64x64.scene.ptd"))
    n = sc.arrays.scene.n_prims
    nodes = np.zeros(2 * n - 1, NODE)
    perm = np.zeros(n, np.int64)
    nn = ctypes.c_int64(0)
    assert lib.pt_host_build_render_tree(None, nodes.ctypes.data, ctypes.byref(nn), perm.ctypes.data) != 0
    assert lib.pt_host_build_render_tree(ctypes.byref(sc.arrays.scene), None, ctypes.byref(nn),
                                         perm.ctypes.data) != 0
    sc.arrays.prim_geom[4] = np.nan
    assert lib.pt_host_build_render_tree(ctypes.byref(sc.arrays.scene), nodes.ctypes.data, ctypes.byref(nn),
                                         perm.ctypes.data) != 0
    assert b"non-finite" in lib.pt_last_error()
