"""Regenerates the committed golden fixtures from the REFERENCE itself.

Runs oracle/_ref/ref_driver (the reference's own CPU path tracer sources,
compiled by oracle/ref/Makefile in the build container; /root/reference is not
available on the GPU box) and stores inputs + outputs as small PTDUMP files:

  c1_<cam>_<W>x<H>.scene.ptd   flattened scene the GPU seam receives (prims in
                               BVH order, BVH nodes, BSDFs, lights, camera)
  c1_<cam>_<W>x<H>_s<spp>_m<depth>_l<ns>_seed<k>.hdr.ptd
                               reference HDR sampleBuffer (float32, y=0 bottom),
                               srand(seed) immediately before start_raytracing, -t 1
  c1_rays.ptd / c1_rays_ref.ptd  ray-query KAT inputs / BVHAccel::intersect answers
  env_sky_64x32{,_half}.exr    synthetic lat-long map written by the reference's
                               tinyexr (ZIP, FLOAT / HALF channels B,G,R)
  env_sky_64x32{,_half}.rgb.ptd  the same files decoded by the reference's load_exr
  <scene>env_<W>x<H>...        scenes / renders with the EnvironmentLight (-e)
  CBspheres_refraction_*       the glass sphere of CBspheres.dae as a <refraction>
                               material (RefractionBSDF, bsdf.cpp:90-111)
  c3proxy_128x128_s64_* / c5proxy_128x128_s64_* / c5bigproxy_128x128_s64_*
                               reference renders of the BASELINE C3 / C5 proxy scenes
                               (scenes.proxy_path(1); scenes.c5_path(2) and c5_path(3) + the env map)
                               at 128x128, 64 spp, two seeds (statistical parity)
  scene_hashes.json             sha256 of every array of the reference's flattened scene for the
                               bunny scenes and the C5 / c5big proxies with their map (1920x1080)
  tocolor_in.ptd / tocolor_ref.ptd
                               HDR edge cases -> HDRImageBuffer::toColor's RGBA8
                               frameBuffer and save_image's flipped rows

Usage: python tests/golden/make_golden.py [--only env|refraction|tocolor|baseline|c5big|c5hashes|highspp]
(needs oracle/_ref/ref_driver)
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from dsgpuraytracing_amd import ptdump  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
C1 = os.path.join(ROOT, "assets", "CBspheres_lambertian.dae")
CAMS = {"default": None, "sphcam": os.path.join(ROOT, "assets", "cam_sphere.info")}

EXTRA_SCENES = ["CBspheres", "CBspheres_lambertian_pointlight", "CBspheres_lambertian_dirlight",
                "CBspheres_lambertian_ambientlight"]

SCENES = [("default", 64, 64), ("sphcam", 96, 64), ("default", 128, 128), ("default", 256, 256)]
RENDERS = [
    # (cam, W, H, spp, depth, ns_area_light, seed)
    ("default", 64, 64, 4, 4, 1, 1),      # exact-parity case (SURVEY §8(c) criterion 1)
    ("sphcam", 96, 64, 3, 4, 2, 7),       # non-square, framed camera, 2 area samples
    ("default", 256, 256, 1, 4, 1, 1),    # BASELINE config C1 (256x256, 1 spp)
    ("default", 128, 128, 64, 4, 1, 1),   # statistical parity pair (noise floor)
    ("default", 128, 128, 64, 4, 1, 2),
]


def scene_name(cam, w, h):
    return f"c1_{cam}_{w}x{h}.scene.ptd"


def hdr_name(cam, w, h, spp, m, l, seed):
    return f"c1_{cam}_{w}x{h}_s{spp}_m{m}_l{l}_seed{seed}.hdr.ptd"


def run(args):
    subprocess.run([REF] + args, check=True, stdout=subprocess.DEVNULL)


ENV_SCENES = [("c1env", C1), ("CBspheresenv", os.path.join(ROOT, "assets", "CBspheres.dae"))]
ENV_RENDERS = [
    # (scene, W, H, spp, depth, ns_area_light, seed)
    ("c1env", 64, 64, 4, 4, 1, 3),
    ("c1env", 64, 64, 4, 4, 2, 4),          # 2 samples per light (area + environment)
    ("CBspheresenv", 64, 64, 4, 4, 1, 3),   # mirror / glass: delta bounces see the map
    ("c1env", 128, 128, 64, 4, 1, 1),       # statistical pair
    ("c1env", 128, 128, 64, 4, 1, 2),
]


def make_env():
    sys.path.insert(0, ROOT)
    from dsgpuraytracing_amd import scenes
    env = scenes.synthetic_envmap(64, 32, seed=3)
    src = os.path.join(HERE, "_tmp_env.ptd")
    ptdump.write(src, {"rgb": env.reshape(-1), "shape": np.array([32, 64, 3], np.int64)})
    for suffix, half in (("", 0), ("_half", 1)):
        exr = os.path.join(HERE, f"env_sky_64x32{suffix}.exr")
        run(["--mode", "exrw", "--in", src, "--out", exr, "--half", str(half)])
        run(["--mode", "exr", "--envmap", exr, "--out", os.path.join(HERE, f"env_sky_64x32{suffix}.rgb.ptd")])
    os.remove(src)
    exr = os.path.join(HERE, "env_sky_64x32.exr")
    for name, dae in ENV_SCENES:
        for w, h in sorted({(r[1], r[2]) for r in ENV_RENDERS if r[0] == name}):
            run([dae, "-w", str(w), "-h", str(h), "--mode", "dump", "--envmap", exr, "--out",
                 os.path.join(HERE, f"{name}_{w}x{h}.scene.ptd")])
    for name, w, h, spp, m, l, seed in ENV_RENDERS:
        dae = dict(ENV_SCENES)[name]
        out = os.path.join(HERE, f"{name}_{w}x{h}_s{spp}_m{m}_l{l}_seed{seed}.hdr.ptd")
        run([dae, "-w", str(w), "-h", str(h), "-s", str(spp), "-m", str(m), "-l", str(l), "--seed", str(seed),
             "--envmap", exr, "--out", out])
        d = ptdump.read(out)
        ptdump.write(out, {"hdr": d["hdr"], "shape": d["shape"]})


def make_refraction():
    """assets/CBspheres_refraction.dae (scenes.refraction_variant) at 64x64
    and 128x128: scene dumps and reference renders."""
    from dsgpuraytracing_amd import scenes
    dae = scenes.refraction_variant(os.path.join(ROOT, "assets", "CBspheres_refraction.dae"))
    name = "CBspheres_refraction"
    for w, h in ((64, 64), (128, 128)):
        run([dae, "-w", str(w), "-h", str(h), "--mode", "dump", "--out", os.path.join(HERE, f"{name}_{w}x{h}.scene.ptd")])
    for w, h, spp, m, l, seed in [(64, 64, 4, 4, 1, 3), (128, 128, 64, 4, 1, 1), (128, 128, 64, 4, 1, 2)]:
        out = os.path.join(HERE, f"{name}_{w}x{h}_s{spp}_m{m}_l{l}_seed{seed}.hdr.ptd")
        run([dae, "-w", str(w), "-h", str(h), "-s", str(spp), "-m", str(m), "-l", str(l), "--seed", str(seed),
             "--out", out])
        d = ptdump.read(out)
        ptdump.write(out, {"hdr": d["hdr"], "shape": d["shape"]})


def make_tocolor():
    """HDR values around every 8-bit code boundary of toColor (image.h:174-189:
    c = pow(s * sqrt(2), 1/2.2), code = (uint32)(min(1, c) * 255)), their float
    neighbours, zeros, denormals, values above 1, +inf and NaN."""
    rng = np.random.default_rng(2201)
    k = np.arange(256, dtype=np.float64)
    bound = (k / 255.0) ** 2.2 / np.sqrt(2.0)
    b32 = bound.astype(np.float32)
    vals = np.concatenate([b32, np.nextafter(b32, np.float32(-1)), np.nextafter(b32, np.float32(2)),
                           np.float32(10.0) ** rng.uniform(-7, 1.5, 2000).astype(np.float32),
                           np.array([0.0, 1e-40, 1e-30, 0.5, 0.7071067, 0.70710677, 0.7071068, 1.0, 3.0, 1e30,
                                     np.inf, np.nan], np.float32)]).astype(np.float32)
    h, w = 48, 64
    n = h * w * 3
    hdr = np.resize(vals, n)
    rng.shuffle(hdr)
    hdr[:vals.size] = vals[: min(vals.size, n)]
    src = os.path.join(HERE, "tocolor_in.ptd")
    ptdump.write(src, {"hdr": hdr, "shape": np.array([h, w, 3], np.int64)})
    run(["--mode", "tocolor", "--in", src, "--out", os.path.join(HERE, "tocolor_ref.ptd")])


def make_baseline_scenes(only=None):
    """The reference's own renders of the C3 and C5 proxies (default camera,
    -m 4 -l 1) at 128x128, 64 spp, seeds 1 and 2; c5bigproxy is C5 at
    BASELINE's "~1M tris" scale (CBbunny_sub3_c5, 1,828,877 primitives)."""
    from dsgpuraytracing_amd import scenes
    for name, dae, env in (("c3proxy", scenes.proxy_path(1), None),
                           ("c5proxy", scenes.c5_path(2), scenes.c5_envmap_path()),
                           ("c5bigproxy", scenes.c5_path(3), scenes.c5_envmap_path())):
        if only and name != only:
            continue
        for seed in (1, 2):
            out = os.path.join(HERE, f"{name}_128x128_s64_m4_l1_seed{seed}.hdr.ptd")
            args = [dae, "-w", "128", "-h", "128", "-s", "64", "-m", "4", "-l", "1", "--seed", str(seed), "--out", out]
            if env:
                args += ["--envmap", env]
            run(args)
            d = ptdump.read(out)
            ptdump.write(out, {"hdr": d["hdr"], "shape": d["shape"]})


# SURVEY.md §8(c) criterion 3's last clause ("at >= 256 spp, the 8x8-box-
# downsampled relative L2 is <= 2%"): the reference's own renders at the spp
# of BASELINE C4 (256) and C5 (512), two seeds each.
# (name, W, H, spp, seeds)
HIGHSPP = [("c1_default", 128, 128, 256, (1, 2)),
           ("c3proxy", 128, 128, 256, (1, 2)),
           ("c5proxy", 64, 64, 512, (1, 2))]


def highspp_name(name, w, h, spp, seed):
    return f"{name}_{w}x{h}_s{spp}_m4_l1_seed{seed}.hdr.ptd"


def make_highspp():
    """Reference renders at >= 256 spp (default camera, -m 4 -l 1, -t 1)."""
    from dsgpuraytracing_amd import scenes
    src = {"c1_default": (C1, None), "c3proxy": (scenes.proxy_path(1), None),
           "c5proxy": (scenes.c5_path(2), scenes.c5_envmap_path())}
    for name, w, h, spp, seeds in HIGHSPP:
        dae, env = src[name]
        for seed in seeds:
            out = os.path.join(HERE, highspp_name(name, w, h, spp, seed))
            args = [dae, "-w", str(w), "-h", str(h), "-s", str(spp), "-m", "4", "-l", "1", "--seed", str(seed),
                    "--out", out]
            if env:
                args += ["--envmap", env]
            run(args)
            d = ptdump.read(out)
            ptdump.write(out, {"hdr": d["hdr"], "shape": d["shape"]})


def main():
    if not os.path.exists(REF):
        sys.exit("oracle/_ref/ref_driver missing: run `make -C oracle/ref` in the build container")
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    if only == "highspp":
        return make_highspp()
    if only == "refraction":
        return make_refraction()
    if only == "tocolor":
        return make_tocolor()
    if only == "baseline":
        return make_baseline_scenes()
    if only == "c5big":
        return make_baseline_scenes("c5bigproxy")
    if only == "c5hashes":
        return make_hashes(c5_only=True)
    make_env()
    if only:
        return
    make_refraction()
    make_tocolor()
    make_baseline_scenes()
    for cam, w, h in SCENES:
        args = [C1, "-w", str(w), "-h", str(h), "--mode", "dump", "--out", os.path.join(HERE, scene_name(cam, w, h))]
        if CAMS[cam]:
            args += ["--cam", CAMS[cam]]
        run(args)
    for cam, w, h, spp, m, l, seed in RENDERS:
        out = os.path.join(HERE, hdr_name(cam, w, h, spp, m, l, seed))
        args = [C1, "-w", str(w), "-h", str(h), "-s", str(spp), "-m", str(m), "-l", str(l), "--seed", str(seed),
                "--out", out]
        if CAMS[cam]:
            args += ["--cam", CAMS[cam]]
        run(args)
        d = ptdump.read(out)
        ptdump.write(out, {"hdr": d["hdr"], "shape": d["shape"]})  # drop the wall time: deterministic file
    # BSDF / light coverage: mirror + glass spheres (CBspheres.dae, the BSDFs of
    # config C5) and point / directional / ambient (hemisphere) light variants.
    for name in EXTRA_SCENES:
        dae = os.path.join(ROOT, "assets", name + ".dae")
        run([dae, "-w", "64", "-h", "64", "--mode", "dump", "--out", os.path.join(HERE, f"{name}_64x64.scene.ptd")])
        renders = [(64, 64, 4, 4, 1, 3)]
        if name == "CBspheres":
            run([dae, "-w", "128", "-h", "128", "--mode", "dump", "--out",
                 os.path.join(HERE, f"{name}_128x128.scene.ptd")])
            renders += [(128, 128, 64, 4, 1, 1), (128, 128, 64, 4, 1, 2)]
        for w, h, spp, m, l, seed in renders:
            out = os.path.join(HERE, f"{name}_{w}x{h}_s{spp}_m{m}_l{l}_seed{seed}.hdr.ptd")
            run([dae, "-w", str(w), "-h", str(h), "-s", str(spp), "-m", str(m), "-l", str(l), "--seed", str(seed),
                 "--out", out])
            d = ptdump.read(out)
            ptdump.write(out, {"hdr": d["hdr"], "shape": d["shape"]})
    # Ray-query KATs on C1: rays from around the box towards random points inside it.
    rng = np.random.default_rng(462)
    n = 2048
    o = rng.uniform(-1.2, 1.2, (n, 3)) + np.array([0.0, 0.75, 0.0])
    tgt = rng.uniform(-1.0, 1.0, (n, 3)) * np.array([1.0, 0.75, 1.0]) + np.array([0.0, 0.75, 0.0])
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    maxt = rng.uniform(0.05, 3.0, n)
    rays = os.path.join(HERE, "c1_rays.ptd")
    ptdump.write(rays, {"ray_o": o.reshape(-1), "ray_d": d.reshape(-1), "ray_maxt": maxt})
    run([C1, "-w", "64", "-h", "64", "--mode", "rays", "--rays", rays, "--out", os.path.join(HERE, "c1_rays_ref.ptd")])
    make_hashes()
    print("golden fixtures written to", HERE)


def make_hashes(c5_only=False):
    """Scene checksums of larger scenes (too big to commit as dumps): the
    reference's own flattened scene, hashed array by array -- the bunny scenes
    and (round 5) the C5 / c5big glass-and-mirror proxies
    with their environment map at 1920x1080.  Merged into scene_hashes.json."""
    sys.path.insert(0, ROOT)
    from dsgpuraytracing_amd import scenes
    path = os.path.join(HERE, "scene_hashes.json")
    hashes = json.load(open(path)) if os.path.exists(path) else {}
    todo = [] if c5_only else [(os.path.join(ROOT, "assets", "CBbunny.dae"), 1024, 1024, None),
                               (scenes.proxy_path(1), 1024, 1024, None), (scenes.proxy_path(1), 1920, 1080, None)]
    todo += [(scenes.c5_path(2), 1920, 1080, scenes.c5_envmap_path()),
             (scenes.c5_path(3), 1920, 1080, scenes.c5_envmap_path())]
    for dae, w, h, env in todo:
        tmp = os.path.join(HERE, "_tmp_scene.ptd")
        args = [dae, "-w", str(w), "-h", str(h), "--mode", "dump", "--out", tmp]
        if env:
            args += ["--envmap", env]
        run(args)
        key = f"{os.path.basename(dae)}@{w}x{h}" + (f"+{os.path.basename(env)}" if env else "")
        hashes[key] = scene_hashes(ptdump.read(tmp))
        os.remove(tmp)
    with open(path, "w") as f:
        json.dump(hashes, f, indent=1, sort_keys=True)


def scene_hashes(d):
    return {k: {"n": int(v.size), "sha256": hashlib.sha256(v.tobytes()).hexdigest()} for k, v in sorted(d.items())}


if __name__ == "__main__":
    main()
