"""CPU checks of bench.py's measurement logic (no GPU): the SURVEY §8(d)
algorithmic-bytes cost model, the roofline views built from the committed PMC
summary, and the agreement of that summary with the rocprofv3 kernel trace
committed beside it (profiles/<round>/)."""
import csv
import json
import os

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_algorithmic_bytes_is_the_survey_cost_model():
    # the C3 counters the round-1 review recomputed by hand: 29.57 GB per launch
    st = {"node_visits": 392_438_744, "tri_tests": 72_187_422, "sphere_tests": 0, "ext_hits": 19_000_062,
          "pixels": 1_048_576}
    want = 64 * 392_438_744 + 48 * 72_187_422 + 4 * 72_187_422 + 36 * 19_000_062 + 12 * 1_048_576
    assert bench.algorithmic_bytes(st) == want
    assert abs(want / 1e9 - 29.57) < 0.01
    # spheres: 16 B per test plus the 4-B primitive index
    st2 = dict(st, tri_tests=0, sphere_tests=10, node_visits=0, ext_hits=0, pixels=0)
    assert bench.algorithmic_bytes(st2) == 10 * (16 + 4)


def test_roofline_views_are_fractions_and_bound_is_the_largest_measured():
    pm = bench.profile_summary("c3")
    assert pm is not None, "profiles/<round>/c3_summary.json missing"
    frame_ms = 1.6
    iso_ms = pm.get("isolated_avg_ms") or 2.0
    alg = 29.5e9
    r = bench.roofline("c3", frame_ms, alg, isolated_ms=iso_ms, pipelined_ms=2.3, lib_sha=pm.get("lib_sha256"))
    views = r["views"]
    for k in ("hbm", "l2", "valu", "algorithmic_cache_served"):
        assert k in views, k
        assert 0.0 < views[k]["frac"] <= 1.0, (k, views[k])
        # the headline fraction is per frame (counts over ms_per_step); the
        # isolated one is the same counts over the kernel's own duration
        assert views[k]["frac_isolated"] == pytest.approx(views[k]["frac"] * frame_ms / iso_ms, rel=1e-3, abs=2e-4)
    measured = {k: views[k]["frac"] for k in ("hbm", "l2", "valu")}
    assert r["bound"] == max(measured, key=measured.get)
    assert r["frac"] == views[r["bound"]]["frac"]
    assert r["duration_ms"] == frame_ms  # no duration above ms_per_step
    assert r["traffic"] == pm["hbm_bytes_per_launch"]
    assert r["pmc_stale"] is False
    assert bench.roofline("c3", frame_ms, alg, lib_sha="0" * 64)["pmc_stale"] is True
    # with a device-code stamp the kernel sha decides (host-only library changes keep the counts)
    if pm.get("kernel_sha256"):
        assert bench.roofline("c3", frame_ms, alg, lib_sha="0" * 64, kernel_sha=pm["kernel_sha256"])["pmc_stale"] is False
        assert bench.roofline("c3", frame_ms, alg, lib_sha=pm["lib_sha256"], kernel_sha="0" * 64)["pmc_stale"] is True
    # HBM bytes from the PMC passes: 2 x FETCH_SIZE + WRITE_SIZE (gfx950 correction), in KB
    assert pm["hbm_bytes_per_launch"] == pytest.approx((2 * pm["fetch_size_kb"] + pm["write_size_kb"]) * 1024,
                                                       rel=1e-6)


def test_pmc_summary_agrees_with_committed_kernel_trace():
    pm = bench.profile_summary("c3")
    src = pm["source"] if os.path.isabs(pm.get("source", "")) else os.path.join(ROOT, pm["source"])
    stats = os.path.join(os.path.dirname(src), "c3_kernel_stats.csv")
    assert os.path.exists(stats), stats
    with open(stats) as f:
        rows = {r["Name"]: r for r in csv.DictReader(f)}
    # the plain render kernel of the summary's round (rounds 1-4: five template
    # arguments; round 5 adds the triangle-only flag; round 6 the frame-batch
    # flag, whose instantiation -- the N = 1 line's frame_batch field -- is not
    # the timed kernel: tools/profile_summary.py timed())
    if pm.get("kernel_name"):  # round 6: the exact timed instantiation (frame batches: the MF one)
        names = [n for n in rows if n == pm["kernel_name"]]
    else:
        names = [n for n in rows if pm.get("kernel", "render_kernel<false, false, false, false, false") in n]
    assert len(names) == 1, names
    avg_ms = float(rows[names[0]]["AverageNs"]) * 1e-6
    assert avg_ms == pytest.approx(pm["avg_ms"], rel=0.02)


def test_committed_bench_lines_keep_the_contract():
    path = os.path.join(ROOT, "profiles", "r3", "bench_c3_default.jsonl")
    with open(path) as f:
        d = json.loads(f.read().strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["metric"] == bench.HEADLINE_METRIC
    assert d["value"] == pytest.approx(1024 * 1024 * 64 / (d["ms_per_step"] * 1e3), rel=0.01)
    assert 0.0 < d["roofline"]["frac"] <= 1.0
    assert d["cpu_baseline"]["kind"] in ("reference", "port") and d["cpu_baseline"]["cores"] >= 1
    for name in ("c3_framed", "c4_single_gpu", "c5_single_gpu", "c3_host_sah", "c3_per_tile", "c3_per_tile_sync"):
        assert d["companions"][name]["value"] > 0, name
    # the roofline's durations: per frame, none above ms_per_step; the isolated
    # kernel time beside it; the PMC summary of the library the line ran
    r = d["roofline"]
    assert r["duration_ms"] == pytest.approx(d["ms_per_step"], rel=1e-3)
    assert r["isolated_kernel_ms"] > 0 and r["frac_isolated"] > 0
    assert d["dist"]["world_size"] == 1


def test_round5_line_reports_one_frames_wall_clock():
    """config.render_time_s is ONE frame's start-to-image
    wall clock (single_frame_ms), not the pipelined interval; the host's share
    of it and an idle synchronize are on the line beside it."""
    path = os.path.join(ROOT, "profiles", "r5", "bench_c3_default.jsonl")
    with open(path) as f:
        d = json.loads(f.read().strip().splitlines()[-1])
    c = d["config"]
    assert c["render_time_s"] == pytest.approx(c["single_frame_ms"] / 1e3, rel=1e-3)
    assert c["wall_clock_frame_ms"] == pytest.approx(c["single_frame_ms"], rel=1e-6)
    assert 0.0 < c["single_frame_api_ms"] < c["single_frame_ms"]
    assert 0.0 < c["sync_floor_ms"] < c["single_frame_ms"]
    # one frame alone takes at least one lone launch, the pipelined step less
    assert c["single_frame_ms"] >= d["roofline"]["isolated_kernel_ms"] >= d["ms_per_step"] * 0.9
    assert d["cpu_baseline_published"]["cores"] == 8


def test_kernel_sha_reads_the_device_code_section():
    from dsgpuraytracing_amd import elfsha, native
    lib = native.LIB_PATH
    code = elfsha.section_bytes(lib, ".hip_fatbin")
    assert len(code) > 100_000  # the gfx950 code objects of every kernel
    assert elfsha.kernel_sha256(lib) == __import__("hashlib").sha256(code).hexdigest()
    assert elfsha.kernel_sha256(lib) != elfsha.file_sha256(lib)
    with pytest.raises(KeyError):
        elfsha.section_bytes(lib, ".no_such_section")


def test_round6_line_reports_the_honest_rates():
    """beside `value`, the line carries the rate of samples
    actually traced (the footprint cull's samples excluded), one frame alone's
    rate (W*H*spp / single_frame_ms) and the isolated launch's VALU-issue
    fraction as roofline.frac_kernel."""
    path = os.path.join(ROOT, "profiles", "r6", "bench_c3_default.jsonl")
    with open(path) as f:
        d = json.loads(f.read().strip().splitlines()[-1])
    c, r = d["config"], d["roofline"]
    whs = c["width"] * c["height"] * c["spp"]
    culled = d["counters"]["culled_samples"]
    assert 0 < culled < whs
    assert d["traced_samples_per_s_M"] == pytest.approx((whs - culled) / (d["ms_per_step"] * 1e3), rel=0.01)
    assert d["traced_samples_per_s_M"] < d["value"]
    assert d["single_frame_Mrays"] == pytest.approx(whs / (c["single_frame_ms"] * 1e3), rel=0.01)
    assert d["single_frame_Mrays"] < d["value"]  # one frame alone does not overlap a neighbour's drain
    assert r["frac_kernel"] == r["views"]["valu"]["frac_isolated"]
    assert 0.0 < r["frac_kernel"] <= 1.0
    assert r["pmc_stale"] is False
    # the node-step census of the STATS launch is on the line
    n = d["launch_counters"]["node_census"]
    assert len(n) == 8 and n[0] > 0 and 0 <= n[1] <= n[0] and n[2] <= n[3]


def test_round6_line_reports_its_frames_per_launch():
    """The C3 line renders its frames eight per launch (frame batches,
    pt_render_frames_device; bit-identical images) and says so -- config and
    launch -- with the launch duration beside the per-frame one; beside it the
    same frames one per launch (the reference's one-frame call)."""
    path = os.path.join(ROOT, "profiles", "r6", "bench_c3_default.jsonl")
    with open(path) as f:
        d = json.loads(f.read().strip().splitlines()[-1])
    assert d["config"]["frames_per_launch"] == 8 == d["launch"]["frames_per_launch"]
    assert d["launch"]["timed_launches"] == -(-d["steps"] // 8)
    one = d["one_frame_per_launch"]
    assert one["frames_per_launch"] == 1 and one["frames"] > 0
    whs = d["config"]["width"] * d["config"]["height"] * d["config"]["spp"]
    assert one["value"] == pytest.approx(whs / (one["ms_per_step"] * 1e3), rel=0.01)
    # the PMC summary counts per frame of the 8-frame launches
    pm = bench.profile_summary("c3")
    assert pm["frames_per_launch"] == 8 and pm["counts_per"] == "frame"
