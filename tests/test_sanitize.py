"""AddressSanitizer + UndefinedBehaviorSanitizer over the host-only code of
libptgpu.so (the reference has no such check; the native host
scene pipeline parses untrusted COLLADA XML and OpenEXR files).

tests/sanitize/host_driver.cpp is linked with csrc/scene_host.cpp, csrc/render_tree.cpp,
csrc/exr_io.cpp, csrc/image_out.cpp and csrc/pt_error.cpp built with
-fsanitize=address,undefined (no recovery) and run over every committed
scene, camera, environment map and the toColor fixture, then over corrupted
copies (truncations at many offsets, byte flips): any sanitizer report fails
the test; ordinary error returns on corrupted input are expected.  The HIP
translation units (pt_api.cpp, the kernels) are covered on the GPU box by
tools/sanitize_gpu.sh (host-side -fsanitize after -Xarch_host)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "dsgpuraytracing_amd", "csrc")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    cxx = shutil.which("g++")
    if not cxx:
        pytest.skip("no g++")
    exe = str(tmp_path_factory.mktemp("san") / "host_driver")
    srcs = [os.path.join(ROOT, "tests", "sanitize", "host_driver.cpp")] + \
        [os.path.join(CSRC, f) for f in ("scene_host.cpp", "render_tree.cpp", "exr_io.cpp", "image_out.cpp", "pt_error.cpp")]
    r = subprocess.run([cxx, "-std=c++17", "-O1", "-g"] + SAN + [f"-I{ROOT}/include", f"-I{CSRC}"] + srcs +
                       ["-lz", "-pthread", "-o", exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


def _run(exe, args, **kw):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    env.update(kw)
    r = subprocess.run([exe] + args, capture_output=True, text=True, env=env, timeout=600)
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    return [ln.split(" ", 1) for ln in r.stdout.splitlines()]


def test_sanitized_host_pipeline_on_fixtures(driver, tmp_path):
    from dsgpuraytracing_amd import scenes
    assets = os.path.join(ROOT, "assets")
    golden = os.path.join(ROOT, "tests", "golden")
    daes = sorted(os.path.join(assets, f) for f in os.listdir(assets) if f.endswith(".dae"))
    daes.append(scenes.proxy_path(1))
    exrs = sorted(os.path.join(golden, f) for f in os.listdir(golden) if f.endswith(".exr"))
    out = _run(driver, daes + exrs + [os.path.join(golden, "tocolor_in.ptd")], PT_SAN_DUMP=str(tmp_path / "d.ptd"))
    assert all(rc == "0" for rc, _ in out), out
    out = _run(driver, ["--cam", os.path.join(assets, "cam_sphere.info"), "--env", exrs[0], scenes.C1_DAE])
    assert all(rc == "0" for rc, _ in out), out


def test_sanitized_host_pipeline_on_corrupted_inputs(driver, tmp_path):
    rng = np.random.default_rng(17)
    files = []
    srcs = [os.path.join(ROOT, "assets", "CBspheres.dae"), os.path.join(ROOT, "assets", "CBspheres_lambertian.dae"),
            os.path.join(ROOT, "tests", "golden", "env_sky_64x32.exr"),
            os.path.join(ROOT, "tests", "golden", "env_sky_64x32_half.exr")]
    for src in srcs:
        data = open(src, "rb").read()
        ext = os.path.splitext(src)[1]
        base = os.path.splitext(os.path.basename(src))[0]
        for k, cut in enumerate(sorted(set(rng.integers(0, len(data), 24).tolist()) | {0, 1, 8, len(data) - 1})):
            p = tmp_path / f"{base}_cut{k}{ext}"
            p.write_bytes(data[:cut])
            files.append(str(p))
        for k in range(24):
            b = bytearray(data)
            for i in rng.integers(0, len(b), 1 + k % 6):
                b[int(i)] = int(rng.integers(0, 256))
            p = tmp_path / f"{base}_flip{k}{ext}"
            p.write_bytes(bytes(b))
            files.append(str(p))
    out = _run(driver, files)
    assert len(out) == len(files)
    assert any(rc != "0" for rc, _ in out)  # the corruptions are detected, not crashed on
