"""The environment light's inverse-CDF search (pt_device.h record_lower_bound,
the kernel's replacement for the two std::lower_bound calls of
EnvironmentLight::importanceSampling, /root/reference/src/static_scene/
environment_light.cpp:69-115) replayed on the host against std::lower_bound
(pt_env_search_check).  The window-halving path runs where a guide bucket's
window spans more than four entries: maps wider than the 1024-bucket guide
table, and nearly flat stretches of a peaky map -- ADVICE r4 found the halved
window returning the whole window's last value as `cur` there."""
import ctypes

import numpy as np

from dsgpuraytracing_amd import native


def _check(rgb, n=200_000, seed=0):
    h, w, _ = rgb.shape
    rng = np.random.default_rng(seed)
    u1 = rng.random(n, dtype=np.float32)
    u2 = rng.random(n, dtype=np.float32)
    # edges of [0, 1): the first and last buckets
    u1[:4] = u2[:4] = np.array([0.0, 1e-9, 0.99999994, 0.5], np.float32)
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    longw = ctypes.c_int64(0)
    bad = native.lib().pt_env_search_check(rgb.ctypes.data, w, h, n, u1.ctypes.data, u2.ctypes.data,
                                           ctypes.byref(longw))
    assert bad >= 0, native.lib().pt_last_error()
    return bad, longw.value


def test_env_search_exact_on_wide_peaky_map():
    # 4096 x 64: four entries per guide bucket along every row, a bright spot
    # over a dim gradient -> long windows everywhere but under the spot
    h, w = 64, 4096
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    rgb = np.repeat((0.01 + 0.001 * x / w)[..., None], 3, axis=2)
    rgb[20:24, 1000:1010] = 500.0
    bad, longw = _check(rgb)
    assert longw > 10_000, "the halving path was not exercised"
    assert bad == 0


def test_env_search_exact_on_small_and_degenerate_maps():
    rng = np.random.default_rng(3)
    for h, w in ((32, 64), (256, 512), (7, 3000), (1, 1), (2, 5000)):
        rgb = rng.random((h, w, 3), dtype=np.float32) ** 8  # peaky
        rgb[:, : w // 3] = 0.0                              # flat (zero) stretch
        bad, _ = _check(rgb, n=50_000, seed=h)
        assert bad == 0, (h, w)
