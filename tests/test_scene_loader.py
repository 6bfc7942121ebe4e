"""Native host scene pipeline (include/ptgpu_scene.h) vs the reference's own
host code: the flattened scene (primitive order, vertex normals, BVH topology
and boxes, BSDFs, lights, camera) must be BIT-IDENTICAL to what
oracle/_ref/ref_driver dumps from the reference sources."""
import hashlib
import json
import os

import numpy as np
import pytest

from dsgpuraytracing_amd import native, ptdump, scene_loader, scenes
from tests.oracle_helpers import golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C1 = os.path.join(ROOT, "assets", "CBspheres_lambertian.dae")


@pytest.mark.parametrize("fixture,w,h,cam", [("c1_default_64x64", 64, 64, None),
                                             ("c1_sphcam_96x64", 96, 64, "cam_sphere.info"),
                                             ("c1_default_128x128", 128, 128, None),
                                             ("c1_default_256x256", 256, 256, None)])
def test_c1_scene_bit_identical_to_reference(fixture, w, h, cam):
    got = scene_loader.load_dae(C1, w, h, os.path.join(ROOT, "assets", cam) if cam else None)
    ref = ptdump.read(golden(f"{fixture}.scene.ptd"))
    assert sorted(got) == sorted(ref)
    for k in ref:
        assert np.array_equal(got[k], ref[k]), k


@pytest.mark.parametrize("name", ["CBspheres", "CBspheres_lambertian_pointlight", "CBspheres_lambertian_dirlight",
                                  "CBspheres_lambertian_ambientlight", "CBspheres_refraction"])
def test_bsdf_and_light_variants_bit_identical(name):
    got = scene_loader.load_dae(os.path.join(ROOT, "assets", name + ".dae"), 64, 64)
    ref = ptdump.read(golden(f"{name}_64x64.scene.ptd"))
    assert sorted(got) == sorted(ref)
    for k in ref:
        assert np.array_equal(got[k], ref[k]), k


@pytest.mark.parametrize("fixture,dae", [("c1env_64x64", "CBspheres_lambertian.dae"),
                                         ("CBspheresenv_64x64", "CBspheres.dae")])
def test_environment_light_scene_bit_identical(fixture, dae):
    """-e map: the environment light is appended last and the map read by the
    native EXR reader equals the reference's (tinyexr) decode."""
    got = scene_loader.load_dae(os.path.join(ROOT, "assets", dae), 64, 64, envmap=golden("env_sky_64x32.exr"))
    ref = ptdump.read(golden(f"{fixture}.scene.ptd"))
    assert sorted(got) == sorted(ref)
    for k in ref:
        assert np.array_equal(got[k], ref[k]), k
    assert got["light_type"][-1] == native.PT_LIGHT_ENVIRONMENT


@pytest.mark.parametrize("key", ["CBbunny.dae@1024x1024", "CBbunny_sub1.dae@1024x1024", "CBbunny_sub1.dae@1920x1080",
                                 "CBbunny_sub2_c5.dae@1920x1080+c5_sky_512x256.exr",
                                 "CBbunny_sub3_c5.dae@1920x1080+c5_sky_512x256.exr"])
def test_bunny_scenes_match_reference_checksums(key):
    """The bunny scenes, and the C5 / c5big glass-and-mirror proxies with their
    environment map (457k / 1.83M primitives: halfedge normals, BVH, the map
    decoded by the native EXR reader), against hashes of the reference's own
    flattened scene (make_golden.py make_hashes: ref_driver --mode dump)."""
    want = json.load(open(golden("scene_hashes.json")))[key]
    name, res = key.split("@")
    res, _, env = res.partition("+")
    w, h = (int(v) for v in res.split("x"))
    dae = {"CBbunny.dae": os.path.join(ROOT, "assets", "CBbunny.dae"), "CBbunny_sub1.dae": scenes.proxy_path(1),
           "CBbunny_sub2_c5.dae": scenes.c5_path(2), "CBbunny_sub3_c5.dae": scenes.c5_path(3)}[name]
    got = scene_loader.load_dae(dae, w, h, envmap=scenes.c5_envmap_path() if env else None)
    assert sorted(got) == sorted(want)
    for k, v in want.items():
        assert got[k].size == v["n"], k
        assert hashlib.sha256(got[k].tobytes()).hexdigest() == v["sha256"], k


def test_bunny_proxy_shape():
    d = scene_loader.load_dae(scenes.proxy_path(1), 64, 64)
    assert len(d["prim_type"]) == 114304 + 12
    ni = d["node_info"].reshape(-1, 4)
    leaves = ni[ni[:, 2] < 0]
    assert leaves[:, 1].sum() == len(d["prim_type"])  # every primitive in exactly one leaf
    assert leaves[:, 1].max() <= 4


def test_loader_errors_are_reported(tmp_path):
    with pytest.raises(native.PtError) as e:
        scene_loader.load_dae(str(tmp_path / "missing.dae"), 8, 8)
    assert e.value.code == native.PT_E_INVALID and "cannot open" in str(e.value)
    bad = tmp_path / "bad.dae"
    bad.write_text("<COLLADA><asset><up_axis>Z_UP</up_axis></asset><scene></COLLADA>")
    with pytest.raises(native.PtError):
        scene_loader.load_dae(str(bad), 8, 8)
    with pytest.raises(native.PtError):
        scene_loader.load_dae(C1, 0, 8)
