// gpu_driver.cpp — TEST DRIVER for the host-AddressSanitizer/UBSan build of
// the whole libptgpu.so source set (HIP translation units included; -fsanitize
// applies to host code only, -Xarch_host) on the GPU box: tools/sanitize_gpu.sh.
// Drives every C-ABI entry point through its success and error paths:
// scene load -> upload (reference BVH and GPU LBVH) -> camera/params ->
// whole-frame, single-tile, ragged, packed and device renders -> ray queries
// -> stats / launch times / wave trace; then malformed scenes, tiles and
// arguments, each of which must be refused with a PT_E_* code.
// usage: gpu_driver <scene.dae> <env.exr> [large_scene.dae]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ptgpu.h"
#include "ptgpu_scene.h"

static int g_bad = 0;
#define OK(x)                                                                   \
  do {                                                                          \
    int rc_ = (x);                                                              \
    if (rc_ != PT_OK) {                                                         \
      std::printf("FAIL %s -> %d (%s)\n", #x, rc_, pt_last_error());            \
      ++g_bad;                                                                  \
    }                                                                           \
  } while (0)
#define REFUSED(x)                                                              \
  do {                                                                          \
    int rc_ = (x);                                                              \
    if (rc_ == PT_OK) {                                                         \
      std::printf("NOT REFUSED %s\n", #x);                                      \
      ++g_bad;                                                                  \
    }                                                                           \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const int W = 96, H = 72;
  pt_host_scene* hs = nullptr;
  OK(pt_host_scene_load(argv[1], W, H, nullptr, &hs));
  pt_scene s;
  pt_camera cam;
  OK(pt_host_scene_view(hs, &s, &cam));
  pt_ctx* c = nullptr;
  OK(pt_create(0, &c));
  std::vector<float> out((size_t)W * H * 3);
  pt_tile whole = {0, 0, W, H}, one = {32, 32, 32, 32}, ragged = {80, 64, 32, 32};
  REFUSED(pt_render_tiles(c, &whole, 1, out.data(), 0));  // no scene yet
  OK(pt_upload_scene(c, &s));
  OK(pt_set_camera(c, &cam));
  pt_params p = {W, H, 4, 4, 1, 7, 0};
  OK(pt_set_params(c, &p));
  OK(pt_render_tiles(c, &whole, 1, out.data(), 0));
  OK(pt_render_tiles(c, &one, 1, out.data(), PT_FLAG_STATS));
  OK(pt_render_tiles(c, &ragged, 1, out.data(), PT_FLAG_REF_COUNTS));
  pt_stats st;
  OK(pt_get_stats(c, &st));
  std::vector<int64_t> trace(1 << 20);
  int64_t nw = 0;
  OK(pt_get_wave_trace(c, trace.data(), (int64_t)trace.size(), &nw));
  float* dev = nullptr;
  if (hipMalloc(&dev, sizeof(float) * W * H * 3) != hipSuccess) return 3;
  pt_tile packed[2] = {{0, 0, 32, 32}, {64, 64, 32, 8}};
  OK(pt_render_tiles_device(c, packed, 2, dev, nullptr, PT_FLAG_PACKED));
  OK(pt_render_tiles_device(c, &whole, 1, dev, nullptr, 0));
  float km[8], rm[8];
  int32_t n = 0;
  OK(pt_get_launch_times(c, km, rm, 8, &n));
  const int64_t R = 1000;
  std::vector<double> o(3 * R), d(3 * R), mt(R);
  for (int64_t i = 0; i < R; ++i) {
    o[3 * i] = -0.5 + i * 1e-3; o[3 * i + 1] = 0.7; o[3 * i + 2] = 3.0;
    d[3 * i] = 0.0; d[3 * i + 1] = -0.05; d[3 * i + 2] = -1.0;
    mt[i] = 1.0 + (double)(i % 7);
  }
  std::vector<int32_t> hit(R), prim(R), any(R);
  std::vector<float> t(R);
  OK(pt_intersect(c, R, o.data(), d.data(), mt.data(), hit.data(), t.data(), prim.data(), any.data()));
  OK(pt_upload_scene_lbvh(c, &s));
  OK(pt_render_tiles(c, &whole, 1, out.data(), 0));
  // malformed inputs: refused, never read out of bounds
  REFUSED(pt_upload_scene(c, nullptr));
  std::vector<int32_t> badb(s.prim_bsdf, s.prim_bsdf + s.n_prims);
  badb[s.n_prims / 2] = s.n_bsdfs;
  pt_scene sb = s;
  sb.prim_bsdf = badb.data();
  REFUSED(pt_upload_scene(c, &sb));
  std::vector<pt_bvh_node> badn(s.nodes, s.nodes + s.n_nodes);
  for (auto& nd : badn)
    if (nd.left >= 0) { nd.left = s.n_nodes + 5; break; }
  pt_scene sn = s;
  sn.nodes = badn.data();
  REFUSED(pt_upload_scene(c, &sn));
  std::vector<pt_bvh_node> badl(s.nodes, s.nodes + s.n_nodes);
  for (auto& nd : badl)
    if (nd.left < 0) { nd.range = s.n_prims + 3; break; }
  pt_scene sl = s;
  sl.nodes = badl.data();
  REFUSED(pt_upload_scene(c, &sl));
  OK(pt_upload_scene(c, &s));  // the context stays usable
  pt_tile neg = {0, 0, -4, 8};
  REFUSED(pt_render_tiles(c, &neg, 1, out.data(), 0));
  REFUSED(pt_render_tiles(c, &whole, 1, nullptr, 0));
  pt_tile big = {0, 0, 64, 32};
  REFUSED(pt_render_tiles_device(c, &big, 1, dev, nullptr, PT_FLAG_PACKED));
  pt_params bp = {W, H, 0, 4, 1, 7, 0};
  REFUSED(pt_set_params(c, &bp));
  pt_camera bc = cam;
  bc.screen_dist = 0;
  REFUSED(pt_set_camera(c, &bc));
  REFUSED(pt_intersect(c, 4, nullptr, d.data(), mt.data(), hit.data(), t.data(), prim.data(), any.data()));
  // environment map scene
  OK(pt_host_scene_set_envmap(hs, argv[2]));
  OK(pt_host_scene_view(hs, &s, &cam));
  OK(pt_upload_scene(c, &s));
  OK(pt_render_tiles(c, &whole, 1, out.data(), 0));
  // a large mesh (optional third argument, e.g. the C3 proxy): the SAH render
  // tree's threaded subtree build, the render over it, the reference-count
  // launch over the caller-order copy, and both trees again
  if (argc > 3) {
    pt_host_scene* hb = nullptr;
    OK(pt_host_scene_load(argv[3], W, H, nullptr, &hb));
    pt_scene sb2;
    pt_camera cb2;
    OK(pt_host_scene_view(hb, &sb2, &cb2));
    OK(pt_upload_scene(c, &sb2));
    OK(pt_set_camera(c, &cb2));
    OK(pt_render_tiles(c, &whole, 1, out.data(), PT_FLAG_STATS));
    OK(pt_render_tiles(c, &whole, 1, out.data(), PT_FLAG_REF_COUNTS));
    OK(pt_intersect(c, 4, o.data(), d.data(), mt.data(), hit.data(), t.data(), prim.data(), any.data()));
    setenv("PT_BVH_BUILD", "ref", 1);
    OK(pt_upload_scene(c, &sb2));
    OK(pt_render_tiles(c, &whole, 1, out.data(), 0));
    unsetenv("PT_BVH_BUILD");
    pt_host_scene_free(hb);
  }
  (void)hipFree(dev);
  OK(pt_destroy(c));
  pt_host_scene_free(hs);
  std::printf("gpu_driver: %d failure(s)\n", g_bad);
  return g_bad ? 1 : 0;
}
