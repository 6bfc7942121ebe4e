"""Deterministic benchmark scenes.

CBdragon.dae (BASELINE configs C3/C4, 100,012 tris) and CBlucy.dae (C5) are
listed in the reference's .MISSING_LARGE_BLOBS and absent here, so the
benchmarks use the proxies SURVEY.md §8(d) specifies: dae/sky/CBbunny.dae with
its bunny geometry ("Mesh-mesh", 28,576 tris) midpoint-subdivided 4:1 per level
(sub1 = 114,304 + 12 box/light tris; sub2 = 457,216 + 12).

Recipe: each triangle (a, b, c) -> (a, ab, ca), (ab, b, bc), (ca, bc, c),
(ab, bc, ca); the edge midpoints are shared through an undirected edge map and
appended after the original vertices in first-use order (ab, bc, ca per
triangle).  The rewritten polylist keeps only the VERTEX input (normals are
recomputed by the halfedge build anyway, src/halfEdgeMesh.h:492-515).
Original vertices keep their exact text; new ones are written with %.7g.
The output is an ordinary .dae that the reference and this package both load.
"""
from __future__ import annotations

import os
import re
from typing import Optional

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASSETS = os.path.join(ROOT, "assets")
C1_DAE = os.path.join(ASSETS, "CBspheres_lambertian.dae")
BUNNY_DAE = os.path.join(ASSETS, "CBbunny.dae")


def _tmp_name(dst: str) -> str:
    """A temporary name private to this process: the ranks of a multi-GPU
    run generate the same scene files concurrently, each writes its own copy
    and os.replace()s it into place (same bytes, atomic)."""
    return f"{dst}.{os.getpid()}.tmp"


def _subdivide_once(pos_tokens, tris):
    """pos_tokens: list of 3-tuples of text tokens; tris: (n,3) int array."""
    pos = np.array([[np.float32(t) for t in p] for p in pos_tokens], dtype=np.float32)
    edge = {}
    new_pos = []
    base = len(pos_tokens)

    def mid(a, b):
        key = (a, b) if a < b else (b, a)
        idx = edge.get(key)
        if idx is None:
            idx = base + len(new_pos)
            edge[key] = idx
            m = (pos[a].astype(np.float64) + pos[b].astype(np.float64)) * 0.5
            new_pos.append(tuple("%.7g" % v for v in m))
        return idx

    out = np.empty((len(tris) * 4, 3), np.int64)
    for i, (a, b, c) in enumerate(tris.tolist()):
        ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
        out[4 * i + 0] = (a, ab, ca)
        out[4 * i + 1] = (ab, b, bc)
        out[4 * i + 2] = (ca, bc, c)
        out[4 * i + 3] = (ab, bc, ca)
    return pos_tokens + new_pos, out


def make_subdivided(src: str, dst: str, levels: int = 1, geometry_id: str = "Mesh-mesh") -> str:
    txt = open(src).read()
    g0 = txt.index(f'<geometry id="{geometry_id}"')
    g1 = txt.index("</geometry>", g0)
    geo = txt[g0:g1]
    m = re.search(r'(<float_array id="[^"]*positions-array" count=")(\d+)(">)([^<]*)(</float_array>)', geo)
    toks = m.group(4).split()
    pos_tokens = [tuple(toks[i:i + 3]) for i in range(0, len(toks), 3)]
    pl = re.search(r"<polylist[^>]*>.*?</polylist>", geo, flags=re.S).group(0)
    inputs = re.findall(r'<input semantic="(\w+)" source="([^"]*)" offset="(\d+)"', pl)
    stride = max(int(o) for _, _, o in inputs) + 1
    voff = [int(o) for s, _, o in inputs if s == "VERTEX"][0]
    vsrc = [src_ for s, src_, _ in inputs if s == "VERTEX"][0]
    vcount = np.array(re.search(r"<vcount>([^<]*)</vcount>", pl).group(1).split(), np.int64)
    if not (vcount == 3).all():
        raise ValueError("subdivision proxy expects a triangle polylist")
    p = np.array(re.search(r"<p>([^<]*)</p>", pl).group(1).split(), np.int64)
    tris = p.reshape(-1, stride)[:, voff].reshape(-1, 3)
    for _ in range(levels):
        pos_tokens, tris = _subdivide_once(pos_tokens, tris)
    mat = re.search(r'material="([^"]*)"', pl).group(1)
    new_pl = (f'<polylist material="{mat}" count="{len(tris)}">\n'
              f'          <input semantic="VERTEX" source="{vsrc}" offset="0"/>\n'
              f'          <vcount>{" ".join(["3"] * len(tris))} </vcount>\n'
              f'          <p>{" ".join(map(str, tris.reshape(-1).tolist()))}</p>\n'
              f'        </polylist>')
    flat = " ".join(" ".join(t) for t in pos_tokens)
    geo2 = geo[:m.start()] + m.group(1) + str(3 * len(pos_tokens)) + m.group(3) + flat + m.group(5) + geo[m.end():]
    geo2 = re.sub(r"<polylist[^>]*>.*?</polylist>", lambda _: new_pl, geo2, count=1, flags=re.S)
    out = txt[:g0] + geo2 + txt[g1:]
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    tmp = _tmp_name(dst)
    with open(tmp, "w") as f:
        f.write(out)
    os.replace(tmp, dst)
    return dst


def proxy_path(levels: int, cache_dir: Optional[str] = None) -> str:
    """Path of CBbunny_sub<levels>.dae, generated on first use."""
    cache_dir = cache_dir or os.path.join(ROOT, "_scenes")
    dst = os.path.join(cache_dir, f"CBbunny_sub{levels}.dae")
    if not os.path.exists(dst) or os.path.getmtime(dst) < os.path.getmtime(__file__):
        make_subdivided(BUNNY_DAE, dst, levels)
    return dst


def synthetic_envmap(width: int = 512, height: int = 256, seed: int = 7) -> np.ndarray:
    """Deterministic lat-long HDR sky (float32, (height, width, 3), row 0 = +y,
    the reference's EnvironmentLight convention theta = (y+0.5)/h*pi): a
    horizon gradient, a darker ground, a small bright sun and low-amplitude
    seeded noise (CBlucy's map is absent)."""
    rng = np.random.RandomState(seed)
    th = (np.arange(height, dtype=np.float64) + 0.5) / height * np.pi       # polar angle from +y
    ph = (np.arange(width, dtype=np.float64) + 0.5) / width * 2.0 * np.pi
    T, Pp = np.meshgrid(th, ph, indexing="ij")
    up = np.cos(T)
    sky = np.stack([0.35 + 0.25 * (1 - up), 0.45 + 0.2 * (1 - up), 0.9 - 0.1 * (1 - up)], -1) * (up > 0)[..., None]
    ground = np.stack([0.18, 0.15, 0.12], -1) * np.ones_like(T)[..., None] * (up <= 0)[..., None]
    # sun at theta = 0.28 pi, phi = 1.3 pi
    sd = np.stack([np.sin(T) * np.cos(Pp), np.cos(T), np.sin(T) * np.sin(Pp)], -1)
    s = np.array([np.sin(0.28 * np.pi) * np.cos(1.3 * np.pi), np.cos(0.28 * np.pi), np.sin(0.28 * np.pi) * np.sin(1.3 * np.pi)])
    cosang = np.clip(sd @ s, -1.0, 1.0)
    sun = 60.0 * np.exp(-(1.0 - cosang) / 0.0015)[..., None] * np.array([1.0, 0.92, 0.8])
    noise = 1.0 + 0.08 * rng.standard_normal((height, width, 1))
    env = (sky + ground) * noise + sun
    return np.ascontiguousarray(np.maximum(env, 0.0).astype(np.float32))


_GLASS_EXTRA = """      <extra>
        <technique profile="CMU462">
          <glass>
            <reflectance>1 1 1</reflectance>
            <transmittance>1 1 1</transmittance>
            <roughness>0</roughness>
            <ior>1.45</ior>
          </glass>
        </technique>
      </extra>
"""

_CHROME_EFFECT = """    <effect id="chrome-effect">
      <profile_COMMON>
        <technique sid="common">
          <phong>
            <diffuse>
              <color sid="diffuse">0.8 0.8 0.8 1</color>
            </diffuse>
          </phong>
        </technique>
      </profile_COMMON>
      <extra>
        <technique profile="CMU462">
          <mirror>
            <reflectance>1 1 1</reflectance>
          </mirror>
        </technique>
      </extra>
    </effect>
"""

_MIRROR_SPHERE_GEOM = """    <geometry id="MirrorSphere-data" name="MirrorSphere">
      <extra>
        <technique profile="CMU462">
          <sphere>
            <radius>.25</radius>
          </sphere>
        </technique>
      </extra>
    </geometry>
"""

_MIRROR_SPHERE_NODE = """      <node id="MirrorSphere" name="MirrorSphere" type="NODE">
        <matrix sid="transform">1 0 0 0.65 0 1 0 0.25 0 0 1 0.45 0 0 0 1</matrix>
        <instance_geometry url="#MirrorSphere-data">
          <bind_material>
            <technique_common>
              <instance_material symbol="chrome" target="#chrome"/>
            </technique_common>
          </bind_material>
        </instance_geometry>
      </node>
"""


def make_c5(levels: int, dst: str) -> str:
    """C5 proxy: CBbunny_sub<levels> with the bunny's
    material switched to <glass> (ior 1.45, the commented template of
    CBspheres_lambertian.dae) and one <mirror> sphere (r = 0.25, resting on
    the floor beside the bunny, in CBspheres.dae's chrome syntax)."""
    txt = open(proxy_path(levels)).read()
    e0 = txt.index('<effect id="Default-effect">')
    e1 = txt.index("</effect>", e0)
    txt = txt[:e1] + _GLASS_EXTRA + "    " + txt[e1:]
    le = txt.index("</library_effects>")
    txt = txt[:le] + _CHROME_EFFECT + "  " + txt[le:]
    lm = txt.index("</library_materials>")
    txt = txt[:lm] + '  <material id="chrome" name="chrome">\n      <instance_effect url="#chrome-effect"/>\n    </material>\n  ' + txt[lm:]
    lg = txt.index("</library_geometries>")
    txt = txt[:lg] + _MIRROR_SPHERE_GEOM + "  " + txt[lg:]
    vs = txt.index("</visual_scene>")
    txt = txt[:vs] + _MIRROR_SPHERE_NODE + "    " + txt[vs:]
    tmp = _tmp_name(dst)
    with open(tmp, "w") as f:
        f.write(txt)
    os.replace(tmp, dst)
    return dst


def c5_path(levels: int = 2, cache_dir: Optional[str] = None) -> str:
    cache_dir = cache_dir or os.path.join(ROOT, "_scenes")
    dst = os.path.join(cache_dir, f"CBbunny_sub{levels}_c5.dae")
    if not os.path.exists(dst) or os.path.getmtime(dst) < os.path.getmtime(__file__):
        make_c5(levels, dst)
    return dst


_REFRACTION_BSDF = """<refraction>
            <transmittance>1 1 1</transmittance>
            <roughness>0</roughness>
            <ior>1.45</ior>
          </refraction>"""


def refraction_variant(dst: str) -> str:
    """CBspheres.dae with its glass sphere's material rewritten as a
    <refraction> material (RefractionBSDF, collada.cpp:893-901, bsdf.cpp:
    90-111; no reference asset uses it): transmittance 1 1 1, roughness 0,
    ior 1.45 -- the glass element's own values.  Everything else is the file
    as shipped."""
    txt = open(os.path.join(ASSETS, "CBspheres.dae")).read()
    g0 = txt.index("<glass>")
    g1 = txt.index("</glass>", g0) + len("</glass>")
    txt = txt[:g0] + _REFRACTION_BSDF + txt[g1:]
    if not os.path.exists(dst) or open(dst).read() != txt:
        tmp = _tmp_name(dst)
        with open(tmp, "w") as f:
            f.write(txt)
        os.replace(tmp, dst)
    return dst


def c5_envmap_path(cache_dir: Optional[str] = None) -> str:
    """The C5 environment map: synthetic_envmap(512, 256, seed=7) as a ZIP OpenEXR."""
    from . import image_io
    cache_dir = cache_dir or os.path.join(ROOT, "_scenes")
    dst = os.path.join(cache_dir, "c5_sky_512x256.exr")
    if not os.path.exists(dst) or os.path.getmtime(dst) < os.path.getmtime(__file__):
        os.makedirs(cache_dir, exist_ok=True)
        tmp = _tmp_name(dst)
        image_io.write_exr(tmp, synthetic_envmap(512, 256, seed=7), "zip")
        os.replace(tmp, dst)
    return dst


if __name__ == "__main__":
    import sys
    for lv in (int(a) for a in sys.argv[1:] or ["1"]):
        print(proxy_path(lv))
