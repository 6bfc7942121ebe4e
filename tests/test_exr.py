"""Native OpenEXR reader (pt_host_load_exr, csrc/exr_io.cpp) vs the reference's
load_exr over tinyexr (src/main.cpp:30-67): the committed fixtures were written
AND decoded by the reference's own tinyexr (tests/golden/make_golden.py).
Host code only: runs without a GPU."""
import numpy as np
import pytest

from dsgpuraytracing_amd import image_io, native, ptdump, scene_loader, scenes
from tests.oracle_helpers import golden


@pytest.mark.parametrize("suffix", ["", "_half"])
def test_native_exr_reader_matches_reference_tinyexr(suffix):
    ref = ptdump.read(golden(f"env_sky_64x32{suffix}.rgb.ptd"))
    got = scene_loader.load_exr(golden(f"env_sky_64x32{suffix}.exr"))
    assert got.shape == tuple(ref["shape"])
    assert np.array_equal(got.reshape(-1), ref["rgb"])


@pytest.mark.parametrize("comp", ["none", "zip"])
@pytest.mark.parametrize("half", [False, True])
def test_exr_writer_round_trip(tmp_path, comp, half):
    env = scenes.synthetic_envmap(40, 23, seed=5)   # 23 rows: a partial last ZIP block
    p = str(tmp_path / "e.exr")
    image_io.write_exr(p, env, comp, half)
    got = scene_loader.load_exr(p)
    want = env.astype(np.float16).astype(np.float32) if half else env
    assert np.array_equal(got, want)


def test_exr_reader_errors(tmp_path):
    bad = tmp_path / "bad.exr"
    bad.write_bytes(b"not an exr file at all")
    with pytest.raises(native.PtError) as e:
        scene_loader.load_exr(str(bad))
    assert e.value.code == native.PT_E_IO
    with pytest.raises(native.PtError):
        scene_loader.load_exr(str(tmp_path / "missing.exr"))
