// host_driver.cpp — TEST DRIVER for the AddressSanitizer / UBSan build of the
// host-only translation units of libptgpu.so (csrc/scene_host.cpp: COLLADA
// parser, halfedge meshes, SAH BVH; csrc/exr_io.cpp: OpenEXR reader;
// csrc/image_out.cpp: toColor; csrc/pt_error.cpp), built and run by
// tests/test_sanitize.py.  Every argument is a file:
//   *.dae  -> pt_host_scene_load at 64x48 (+ the .info camera given with
//             --cam, + the environment map given with --env), view, dump,
//             free; a non-zero return is fine for corrupted inputs, a
//             sanitizer report is not
//   *.exr  -> pt_host_load_exr
//   *.ptd  -> pt_to_color of its "hdr" record (tocolor fixture)
// Prints one line per file: "<rc> <path>".
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ptdump.h"
#include "ptgpu.h"
#include "ptgpu_scene.h"

static bool ends_with(const std::string& s, const char* suf) {
  size_t n = std::strlen(suf);
  return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}

int main(int argc, char** argv) {
  const char* cam = nullptr;
  const char* env = nullptr;
  const char* dump = std::getenv("PT_SAN_DUMP");
  int failures = 0;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--cam" && i + 1 < argc) { cam = argv[++i]; continue; }
    if (a == "--env" && i + 1 < argc) { env = argv[++i]; continue; }
    int rc = 0;
    if (ends_with(a, ".dae")) {
      pt_host_scene* hs = nullptr;
      rc = pt_host_scene_load(a.c_str(), 64, 48, cam, &hs);
      if (rc == PT_OK && env) rc = pt_host_scene_set_envmap(hs, env);
      if (rc == PT_OK) {
        pt_scene s;
        pt_camera c;
        rc = pt_host_scene_view(hs, &s, &c);
        double acc = 0;  // touch every array the view hands out
        for (int64_t k = 0; rc == PT_OK && k < s.n_prims; ++k)
          acc += s.prim_type[k] + s.prim_bsdf[k] + s.prim_geom[9 * k + 8] + s.prim_norm[9 * k + 8];
        for (int64_t k = 0; rc == PT_OK && k < s.n_nodes; ++k) acc += s.nodes[k].bb_max[2] + (double)s.nodes[k].right;
        if (rc == PT_OK && dump) rc = pt_host_scene_dump(hs, dump);
        if (rc == PT_OK) {  // the render tree pt_upload_scene builds (threaded for big meshes)
          std::vector<pt_bvh_node> tree((size_t)(2 * s.n_prims - 1));
          std::vector<int64_t> perm((size_t)s.n_prims);
          int64_t nn = 0;
          rc = pt_host_build_render_tree(&s, tree.data(), &nn, perm.data());
          for (int64_t k = 0; rc == PT_OK && k < nn; ++k) acc += tree[(size_t)k].bb_min[0] + (double)perm[(size_t)(k % s.n_prims)];
        }
        if (acc == 12345.678) std::puts("");
      }
      pt_host_scene_free(hs);
    } else if (ends_with(a, ".exr")) {
      int32_t w = 0, h = 0;
      float* rgb = nullptr;
      rc = pt_host_load_exr(a.c_str(), &w, &h, &rgb);
      if (rc == PT_OK) {
        double acc = 0;
        for (int64_t k = 0; k < (int64_t)w * h * 3; ++k) acc += rgb[k];
        if (acc == 12345.678) std::puts("");
      }
      pt_host_free(rgb);
    } else if (ends_with(a, ".ptd")) {
      std::vector<ptdump::Record> R;
      std::vector<float> hdr;
      std::vector<int64_t> shape;
      if (!ptdump::read_all(a.c_str(), R) || !ptdump::get(R, "hdr", hdr) || !ptdump::get(R, "shape", shape)) {
        rc = -100;
      } else {
        std::vector<uint32_t> frame((size_t)(shape[0] * shape[1]));
        rc = pt_to_color(hdr.data(), (int32_t)shape[1], (int32_t)shape[0], -5, -5, 1 << 20, 1 << 20, frame.data());
      }
    } else {
      rc = -101;
      ++failures;
    }
    std::printf("%d %s\n", rc, a.c_str());
  }
  return failures ? 3 : 0;
}
