"""Parity at BASELINE.json's full sizes.

C1 (256x256, 1 spp) and C2 (512x512, 16 spp) are cheap for the oracle, so the
whole HIP frame is compared with the whole restatement frame (counter RNG, the
same draws in the same order).  For C3 (1024x1024, 64 spp), C4 (1920x1080,
256 spp) and C5 (1920x1080, 512 spp) the GPU renders the whole frame and the
restatement renders a spread of sampled 32x32 tiles of it, which must match
near-exactly; the size-independent properties of the whole frame are checked
as well: finite and non-negative radiance, determinism, and that a tile split
(the multi-GPU strong split) reassembles the frame bit for bit.

The sampled tiles are chosen FROM THE ORACLE, never by hand: a 1-spp
restatement render of the whole frame (C3: 0.15 s, C5: 1 s on 8 threads) gives
every tile's coverage.  Two kinds are taken, each at evenly spaced ranks of
its candidates: LIT tiles (every pixel saw radiance) and MIXED tiles (both
black and lit pixels: the silhouettes of the scene box and of the geometry,
where fp32-vs-fp64 decisions, the integer-ulp origin offsets and the screen
footprint's 1-px margin act).  The precondition (every chosen reference tile
is lit somewhere) is asserted before the GPU render.  The screen-footprint
cull of the headline frame is also checked against tracing every sample, at
full size (C3 at 64 spp, C4 at a reduced spp).

Tolerance (SURVEY.md §8(c) criterion 2), for every config: >= 99.5% of
pixels within 1e-3 relative and the (sampled-tile) image mean within 0.1%.
Measured on the box: C1 100%, C2 99.995%, C3 99.988%,
C4 99.935%, C5 99.902% of pixels; mean differences 2e-6 .. 1.3e-5.
"""
import os

import numpy as np
import pytest

from dsgpuraytracing_amd import ptdump, scene_loader, scenes
from dsgpuraytracing_amd.dist import shard_tiles
from dsgpuraytracing_amd.pathtracer import Device, Scene, tile_fifo

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
THREADS = max(1, min(16, len(os.sched_getaffinity(0))))  # the host threads a GPU's job owns (16 on the box)

WORKLOADS = {
    # name: (dae, envmap, W, H, spp)
    "c1": (scenes.C1_DAE, None, 256, 256, 1),
    "c2": (scenes.C1_DAE, None, 512, 512, 16),
    "c3": ("proxy1", None, 1024, 1024, 64),
    "c4": ("proxy1", None, 1920, 1080, 256),
    "c5": ("c5", "c5env", 1920, 1080, 512),
    # C5 at BASELINE's "~1M tris" scale: CBbunny_sub3_c5 (1,828,877 primitives)
    "c5big": ("c5big", "c5env", 1920, 1080, 512),
}


def _workload(name):
    dae, env, w, h, spp = WORKLOADS[name]
    if dae == "proxy1":
        dae = scenes.proxy_path(1)
    elif dae == "c5":
        dae = scenes.c5_path(2)
    elif dae == "c5big":
        dae = scenes.c5_path(3)
    if env == "c5env":
        env = scenes.c5_envmap_path()
    return dae, env, w, h, spp


def _device(dae, envmap, w, h, spp, seed=1, dump=None):
    """dump: the scene already flattened (scene_loader.dump_dae) -- large
    scenes are loaded once for both the oracle and the GPU."""
    sc = Scene.from_dump(dump) if dump else Scene.from_dae(dae, w, h, envmap=envmap)
    dev = Device(0)
    dev.upload_scene(sc)
    dev.set_camera(sc.camera)
    dev.set_params(w, h, spp, 4, 1, seed)
    return dev


def near_exact(a, b):
    diff = np.abs(a - b).max(axis=-1)
    scale = np.maximum(1.0, np.abs(b).max(axis=-1))
    return float((diff <= 1e-3 * scale).mean())


def without_environment(dump, out):
    """The scene of `dump` without its EnvironmentLight: camera rays that miss
    the scene are black here, so the mixed tiles of this scene are the
    silhouettes of the geometry against the environment."""
    d = ptdump.read(dump)
    keep = d["light_type"] != 4
    nl = len(d["light_type"])
    for key in ("light_type", "light_rad", "light_geom", "light_area"):
        per = d[key].size // nl
        d[key] = d[key].reshape(nl, per)[keep].reshape(-1)
    d.pop("env_shape", None)
    d.pop("env_rgb", None)
    ptdump.write(out, d)
    return out


def oracle_tiles(restate, dump, w, h, k, kind="lit", seed=1):
    """k 32x32 tiles of the frame at evenly spaced ranks of the tile FIFO
    order, chosen from a 1-spp restatement render: kind "lit" = full tiles
    every pixel of which receives radiance; "mixed" = tiles (ragged edge
    tiles included) holding both black and lit pixels.  For a scene with an
    environment light pass its dump without_environment() for the mixed
    tiles: the silhouettes against the environment."""
    one, _ = restate.render(dump, w, h, 1, 4, 1, seed, rng_mode=1, threads=THREADS)
    cand = []
    for x, y, _, _ in tile_fifo(w, h):
        lit = one[y:y + 32, x:x + 32].max(axis=2) > 0
        if kind == "lit" and x + 32 <= w and y + 32 <= h and lit.all():
            cand.append((x, y))
        elif kind == "mixed" and lit.any() and not lit.all():
            cand.append((x, y))
    assert len(cand) >= k, f"only {len(cand)} {kind} tiles"
    pick = np.linspace(0, len(cand) - 1, k).round().astype(int)
    return [cand[i] for i in pick]


def lit_tiles(restate, dump, w, h, k, seed=1):
    return oracle_tiles(restate, dump, w, h, k, "lit", seed)


@pytest.mark.parametrize("name", ["c1", "c2"])
def test_fullframe_near_exact_vs_oracle(tmp_path, restate, name):
    dae, envmap, w, h, spp = _workload(name)
    dump = str(tmp_path / f"{name}.ptd")
    scene_loader.dump_dae(dae, w, h, dump, envmap=envmap)
    ref, _ = restate.render(dump, w, h, spp, 4, 1, 1, rng_mode=1, threads=THREADS)
    assert ref.mean() > 0
    dev = _device(dae, envmap, w, h, spp)
    img = np.zeros((h, w, 3), np.float32)
    dev.render_tiles(tile_fifo(w, h), img)
    assert np.isfinite(img).all() and (img >= 0).all()
    close = near_exact(img, ref)
    rel_mean = abs(img.mean() - ref.mean()) / ref.mean()
    print(f"{name}: {close * 100:.3f}% pixels within 1e-3, image-mean rel diff {rel_mean:.2e}")
    assert close >= 0.995, close
    assert rel_mean <= 1e-3, rel_mean


# (name, lit tiles, mixed tiles, per-pixel near-exact fraction: SURVEY's 99.5% pooled
# per kind, and SURVEY's 99.5% in every single tile too -- TILE_FLOOR -- except the
# tiles named in TILE_EXCEPTIONS).  C5 has an environment light: no pixel is black,
# so its mixed tiles are those of the scene without the environment light -- the
# silhouettes of the box and bunny against the sky.
TILE_FLOOR = 0.995
# Sampled tiles below 99.5%, each with its sample-by-sample census
# (tools/silhouette_samples.py: every off pixel's difference equals the sum of
# its differing samples' differences / spp, so nothing else differs):
#  * C4 (1088, 192), 0.9883 on the box: 12 off pixels, each differing in ONE or
#    two of 256 samples whose path took another turn at a silhouette (fp32 vs
#    fp64 hit decisions at grazing incidence; profiles/r4/silhouette_c4_1088_192.txt);
#  * C5 (800, 416), 0.9932: 7 off pixels at the glass bunny's edge against the
#    sky, each differing in 4-12 of 512 samples by 0.1-3% of the sample -- fp32
#    drift of refracted directions that look the environment map up a little
#    elsewhere, no discrete decision and no sign bias (profiles/r6/silhouette_c5_800_416.txt).
TILE_EXCEPTIONS = {
    ("c4", (1088, 192)): 0.985,
    ("c5", (800, 416)): 0.99,
}


@pytest.mark.parametrize("name,k,k_mixed,min_close", [
    ("c3", 8, 6, 0.995),
    ("c4", 6, 6, 0.995),
    ("c5", 3, 3, 0.995),
    ("c5big", 2, 2, 0.995),
])
def test_fullsize_sampled_tiles_match_oracle(tmp_path, restate, name, k, k_mixed, min_close):
    dae, envmap, w, h, spp = _workload(name)
    dump = str(tmp_path / f"{name}.ptd")
    scene_loader.dump_dae(dae, w, h, dump, envmap=envmap)
    tiles = lit_tiles(restate, dump, w, h, k)
    sil = without_environment(dump, str(tmp_path / f"{name}_noenv.ptd")) if envmap else dump
    mixed = oracle_tiles(restate, sil, w, h, k_mixed, "mixed") if k_mixed else []
    tw = (w + 31) // 32
    refs = []
    for x, y in tiles + mixed:   # the oracle first: its precondition is checked before the GPU runs
        t = (y // 32) * tw + x // 32
        ref, _ = restate.render(dump, w, h, spp, 4, 1, 1, rng_mode=1, threads=THREADS, tile_begin=t, tile_end=t + 1)
        b = ref[y:y + 32, x:x + 32]
        assert b.mean() > 0, (x, y)
        refs.append(b)
    dev = _device(dae, envmap, w, h, spp, dump=dump)
    img = np.zeros((h, w, 3), np.float32)
    dev.render_tiles(tile_fifo(w, h), img)
    assert np.isfinite(img).all() and (img >= 0).all()
    for kind, sel, rf in (("lit", tiles, refs[:len(tiles)]), ("mixed", mixed, refs[len(tiles):])):
        if not sel:
            continue
        got = [img[y:y + 32, x:x + 32] for x, y in sel]
        closes = [near_exact(a, b) for a, b in zip(got, rf)]
        gflat = np.concatenate([a.reshape(-1, 3) for a in got])
        rflat = np.concatenate([b.reshape(-1, 3) for b in rf])
        close = near_exact(gflat, rflat)
        rel_mean = abs(gflat.mean() - rflat.mean()) / rflat.mean()
        # the black pixels of mixed tiles are black on both sides (exact)
        black = rflat.max(axis=1) == 0
        print(f"{name} {kind}: tiles {sel}\n  per-tile {np.round(closes, 4).tolist()}\n"
              f"  {close * 100:.3f}% pixels within 1e-3, sampled-tile mean rel diff {rel_mean:.2e}, "
              f"{int(black.sum())} black reference pixels")
        assert close >= min_close, (kind, closes)
        for (x, y), c in zip(sel, closes):
            assert c >= TILE_EXCEPTIONS.get((name, (x, y)), TILE_FLOOR), (kind, (x, y), c)
        assert rel_mean <= 1e-3, (kind, rel_mean)
        if black.any():
            assert (gflat[black] == 0).mean() >= min_close, kind


@pytest.mark.parametrize("name,spp", [("c3", 64), ("c4", 16)])
def test_footprint_cull_exact_at_full_size(monkeypatch, name, spp):
    """The headline's default camera leaves most of the frame outside the
    scene box's screen footprint (pt_api.cpp screen_footprint): those samples
    are not traced (camera.cpp:113-129 rays that miss the root box see
    nothing, pathtracer.cpp:421-426).  The culled frame must equal the frame
    traced sample by sample (PT_NO_FOOTPRINT_CULL=1) bit for bit, edges and
    silhouettes included; C4 at a reduced spp (the cull does not depend on it)."""
    dae, envmap, w, h, _ = _workload(name)
    dev = _device(dae, envmap, w, h, spp, seed=5)
    monkeypatch.delenv("PT_NO_FOOTPRINT_CULL", raising=False)
    culled = np.zeros((h, w, 3), np.float32)
    dev.render_tiles(tile_fifo(w, h), culled, stats=True)
    st = dev.stats()
    monkeypatch.setenv("PT_NO_FOOTPRINT_CULL", "1")
    traced = np.zeros_like(culled)
    dev.render_tiles(tile_fifo(w, h), traced, stats=True)
    st2 = dev.stats()
    print(f"{name}: culled {st['culled_samples']} of {w * h * spp} samples; camera rays {st['camera_rays']} "
          f"vs {st2['camera_rays']} traced")
    assert st["culled_samples"] > 0 and st2["culled_samples"] == 0
    assert st["camera_rays"] + st["culled_samples"] == st2["camera_rays"]
    assert np.array_equal(culled, traced)
    # ... and the same for the plain (counter-free) build
    plain_traced = np.zeros_like(culled)
    dev.render_tiles(tile_fifo(w, h), plain_traced)
    monkeypatch.delenv("PT_NO_FOOTPRINT_CULL")
    plain = np.zeros_like(culled)
    dev.render_tiles(tile_fifo(w, h), plain)
    assert np.array_equal(plain, plain_traced)
    assert np.array_equal(plain, culled)
    assert culled.mean() > 0
    # the reported footprint (pt_stats.footprint; bench.py's weak-scaling
    # reduce carries only its rows): everything outside it is exactly 0 in the
    # TRACED frame, and the rectangle is not the whole frame here
    x0, y0, x1, y1 = st["footprint"]
    assert 0 <= x0 <= x1 < w and 0 <= y0 <= y1 < h
    assert (x1 - x0 + 1) * (y1 - y0 + 1) < w * h
    outside = np.ones((h, w), bool)
    outside[y0:y1 + 1, x0:x1 + 1] = False
    assert not traced[outside].any()
    assert st2["footprint"] == [0, 0, w - 1, h - 1]


def test_c3_fullsize_deterministic_and_split():
    dae, envmap, w, h, spp = _workload("c3")
    dev = _device(dae, envmap, w, h, spp, seed=3)
    full = np.zeros((h, w, 3), np.float32)
    dev.render_tiles(tile_fifo(w, h), full)
    again = np.zeros_like(full)
    dev.render_tiles(tile_fifo(w, h), again)
    assert np.array_equal(full, again)
    parts = np.zeros_like(full)
    for r in range(3):  # the strong multi-GPU split, one share at a time
        p = np.zeros_like(full)
        dev.render_tiles(shard_tiles(tile_fifo(w, h), r, 3, "diag"), p)
        parts += p
    assert np.array_equal(parts, full)


def test_c4_fullsize_eight_way_split_bit_identical():
    """BASELINE C4's multi-GPU split: the 8 diagonal tile shards, rendered one
    share at a time, reassemble the 1-GPU frame bit for bit."""
    dae, envmap, w, h, _ = _workload("c4")
    spp = 16   # the split property does not depend on spp; 16 keeps the test short
    dev = _device(dae, envmap, w, h, spp, seed=4)
    full = np.zeros((h, w, 3), np.float32)
    dev.render_tiles(tile_fifo(w, h), full)
    parts = np.zeros_like(full)
    for r in range(8):
        p = np.zeros_like(full)
        dev.render_tiles(shard_tiles(tile_fifo(w, h), r, 8, "diag"), p)
        parts += p
    assert np.array_equal(parts, full)
    assert full.mean() > 0


def test_c3_small_launch_shape_never_changes_values(monkeypatch):
    """The small-launch shape (pt_api.cpp launch: a strong split's share has
    few work slots per lane, so it claims 64 slots at a time and, queued
    behind other frames, runs on half the resident grid with up to four
    frames in flight) changes only which wave renders which slot: the C3
    frame's 8-way diagonal shares, queued back to back on one stream (the
    bench's N > 1 pattern), reassemble the whole frame -- a large launch --
    bit for bit, and equal the shares rendered with the shape turned off."""
    import torch
    dae, envmap, w, h, spp = _workload("c3")
    dev = _device(dae, envmap, w, h, spp, seed=6)
    stream = torch.cuda.Stream(device=0)
    whole = np.asarray(tile_fifo(w, h), np.int32).reshape(-1, 4)
    full = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda:0")
    dev.render_tiles_device(whole, full.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()

    def split(n_rounds=2):
        parts = [torch.zeros_like(full) for _ in range(8)]
        for _ in range(n_rounds):  # queued: every launch after the first finds the GPU busy
            for r in range(8):
                share = np.asarray(shard_tiles(tile_fifo(w, h), r, 8, "diag"), np.int32).reshape(-1, 4)
                dev.render_tiles_device(share, parts[r].data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        return torch.stack(parts).sum(0)

    monkeypatch.delenv("PT_SMALL_LAUNCH", raising=False)
    small = split()
    assert torch.equal(small, full)
    monkeypatch.setenv("PT_SMALL_LAUNCH", "0")
    assert torch.equal(split(), full)
    assert float(full.mean()) > 0
