// render_tree.cpp -- the render tree pt_upload_scene builds over the handed-over
// primitives (host only).  C ABI: pt_host_build_render_tree
// (include/ptgpu_scene.h), called by pt_api.cpp's upload and by the CPU tests.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ptgpu.h"
#include "../../include/ptgpu_scene.h"
#include "pt_error.h"

namespace {

// ---- Own binned-SAH binary tree over the scene's primitives (PT_BVH_BUILD=sah).
// The traversal result is the nearest hit whatever the tree, so the tree is
// free to follow this kernel's cost model instead of the reference's builder
// (bvh.cpp:21-178: 32 buckets over the node box, always split down to <= 4).
// Here: PT_SAH_BINS buckets over the CENTROID bounds, per-axis sweeps, and a
// leaf wherever the SAH says a split no longer pays (C_trav = 1 per binary
// node, C_isect = PT_SAH_CI per primitive), at most PT_SAH_LEAF primitives.
// Output in the reference's pt_bvh_node format (pre-order, ranges over the
// permuted primitive order `perm`: new index -> uploaded index), so the
// BVH4 collapse below is shared with the reference-tree path.
void build_sah_tree(const pt_scene* s, std::vector<pt_bvh_node>& out, std::vector<int64_t>& perm) {
  const int64_t n = s->n_prims;
  const int bins = std::getenv("PT_SAH_BINS") ? std::max(2, std::atoi(std::getenv("PT_SAH_BINS"))) : 128;
  const double ci = std::getenv("PT_SAH_CI") ? std::atof(std::getenv("PT_SAH_CI")) : 1.0;
  const int64_t max_leaf = std::getenv("PT_SAH_LEAF") ? std::max(1, std::min(8, std::atoi(std::getenv("PT_SAH_LEAF")))) : 4;
  std::vector<double> lo((size_t)n * 3), hi((size_t)n * 3), cen((size_t)n * 3);
  for (int64_t i = 0; i < n; ++i) {
    const double* g = s->prim_geom + 9 * i;
    for (int k = 0; k < 3; ++k) {
      double a, b;
      if (s->prim_type[i] == PT_PRIM_TRIANGLE) {
        a = std::min({g[k], g[3 + k], g[6 + k]});
        b = std::max({g[k], g[3 + k], g[6 + k]});
      } else {
        a = g[k] - std::fabs(g[3]);
        b = g[k] + std::fabs(g[3]);
      }
      lo[3 * i + k] = a;
      hi[3 * i + k] = b;
      cen[3 * i + k] = 0.5 * (a + b);
    }
  }
  auto half_area = [](const double* a, const double* b) {
    const double dx = b[0] - a[0], dy = b[1] - a[1], dz = b[2] - a[2];
    return dx * dy + dy * dz + dz * dx;
  };
  perm.resize((size_t)n);
  for (int64_t i = 0; i < n; ++i) perm[(size_t)i] = i;
  out.clear();
  struct Task { int64_t node, start, count; };
  auto make_node = [&](std::vector<pt_bvh_node>& o, int64_t start, int64_t count) {
    pt_bvh_node d{};
    for (int k = 0; k < 3; ++k) {
      d.bb_min[k] = INFINITY;
      d.bb_max[k] = -INFINITY;
    }
    for (int64_t j = start; j < start + count; ++j) {
      const int64_t p = perm[(size_t)j];
      for (int k = 0; k < 3; ++k) {
        d.bb_min[k] = std::min(d.bb_min[k], lo[3 * p + k]);
        d.bb_max[k] = std::max(d.bb_max[k], hi[3 * p + k]);
      }
    }
    d.start = start;
    d.range = count;
    d.left = d.right = -1;
    o.push_back(d);
    return (int64_t)o.size() - 1;
  };
  struct Bin { double lo[3], hi[3]; int64_t n; };
  // Builds the subtree of task `t0` into `o` (t0.node indexes `o`); tasks of
  // fewer than `defer_below` primitives go to `deferred` instead (the
  // parallel phase), when given.  Touches only perm[t0.start, +t0.count).
  auto build = [&](std::vector<pt_bvh_node>& o, Task t0, int64_t defer_below, std::vector<Task>* deferred) {
    std::vector<Bin> bn((size_t)bins);
    std::vector<double> rcost((size_t)bins);
    std::vector<Task> st = {t0};
    while (!st.empty()) {
      const Task t = st.back();
      st.pop_back();
      if (t.count <= 1) continue;
      if (deferred && t.count < defer_below) {
        deferred->push_back(t);
        continue;
      }
      double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
      for (int64_t j = t.start; j < t.start + t.count; ++j)
        for (int k = 0; k < 3; ++k) {
          clo[k] = std::min(clo[k], cen[3 * perm[(size_t)j] + k]);
          chi[k] = std::max(chi[k], cen[3 * perm[(size_t)j] + k]);
        }
      const double area = half_area(o[(size_t)t.node].bb_min, o[(size_t)t.node].bb_max);
      double best = INFINITY;
      int best_axis = -1, best_split = 0;
      for (int k = 0; k < 3; ++k) {
        if (!(chi[k] > clo[k])) continue;
        const double scale = bins / (chi[k] - clo[k]);
        for (Bin& b : bn) {
          b.n = 0;
          for (int q = 0; q < 3; ++q) {
            b.lo[q] = INFINITY;
            b.hi[q] = -INFINITY;
          }
        }
        for (int64_t j = t.start; j < t.start + t.count; ++j) {
          const int64_t p = perm[(size_t)j];
          const int b = std::min(bins - 1, (int)((cen[3 * p + k] - clo[k]) * scale));
          Bin& B = bn[(size_t)b];
          B.n++;
          for (int q = 0; q < 3; ++q) {
            B.lo[q] = std::min(B.lo[q], lo[3 * p + q]);
            B.hi[q] = std::max(B.hi[q], hi[3 * p + q]);
          }
        }
        // right sweep: cost of bins [b, bins)
        double rl[3] = {INFINITY, INFINITY, INFINITY}, rh[3] = {-INFINITY, -INFINITY, -INFINITY};
        int64_t rn = 0;
        for (int b = bins - 1; b > 0; --b) {
          const Bin& B = bn[(size_t)b];
          rn += B.n;
          for (int q = 0; q < 3; ++q) {
            rl[q] = std::min(rl[q], B.lo[q]);
            rh[q] = std::max(rh[q], B.hi[q]);
          }
          rcost[(size_t)b] = rn ? half_area(rl, rh) * (double)rn : 0.0;
        }
        double ll[3] = {INFINITY, INFINITY, INFINITY}, lh[3] = {-INFINITY, -INFINITY, -INFINITY};
        int64_t ln = 0;
        for (int b = 0; b < bins - 1; ++b) {  // split between bin b and b+1
          const Bin& B = bn[(size_t)b];
          ln += B.n;
          for (int q = 0; q < 3; ++q) {
            ll[q] = std::min(ll[q], B.lo[q]);
            lh[q] = std::max(lh[q], B.hi[q]);
          }
          if (ln == 0 || ln == t.count) continue;
          const double c = half_area(ll, lh) * (double)ln + rcost[(size_t)b + 1];
          if (c < best) {
            best = c;
            best_axis = k;
            best_split = b + 1;
          }
        }
      }
      const double split_cost = 1.0 + ci * best / std::max(area, 1e-300);
      const double leaf_cost = ci * (double)t.count;
      int64_t mid;
      if (best_axis < 0) {  // coincident centroids
        if (t.count <= max_leaf) continue;
        mid = t.start + t.count / 2;
      } else {
        if (t.count <= max_leaf && leaf_cost <= split_cost) continue;
        const double scale = bins / (chi[best_axis] - clo[best_axis]);
        auto it = std::partition(perm.begin() + t.start, perm.begin() + t.start + t.count, [&](int64_t p) {
          return std::min(bins - 1, (int)((cen[3 * p + best_axis] - clo[best_axis]) * scale)) < best_split;
        });
        mid = (int64_t)(it - perm.begin());
      }
      const int64_t l = make_node(o, t.start, mid - t.start);
      const int64_t r = make_node(o, mid, t.start + t.count - mid);
      o[(size_t)t.node].left = l;
      o[(size_t)t.node].right = r;
      st.push_back({r, mid, t.start + t.count - mid});
      st.push_back({l, t.start, mid - t.start});
    }
  };
  // The top of the tree on this thread until the open subtrees are small,
  // then the subtrees on a pool of host threads (disjoint primitive ranges,
  // private node arrays), spliced in afterwards.  The result does not depend
  // on the thread count: every subtree is built by the same sequential code.
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const int threads = std::getenv("PT_BUILD_THREADS") ? std::max(1, std::atoi(std::getenv("PT_BUILD_THREADS")))
                                                      : (int)std::min(16u, hw);
  std::vector<Task> deferred;
  const int64_t defer_below = threads > 1 && n >= 8192 ? std::max<int64_t>(2048, n / (8 * threads)) : 0;
  build(out, Task{make_node(out, 0, n), 0, n}, defer_below, defer_below ? &deferred : nullptr);
  if (!deferred.empty()) {
    std::vector<std::vector<pt_bvh_node>> sub(deferred.size());
    std::atomic<size_t> next{0};
    auto worker = [&]() {
      for (size_t i; (i = next.fetch_add(1)) < deferred.size();) {
        sub[i].push_back(out[(size_t)deferred[i].node]);  // the subtree root as local node 0
        build(sub[i], Task{0, deferred[i].start, deferred[i].count}, 0, nullptr);
      }
    };
    std::vector<std::thread> pool;
    for (int k = 1; k < threads; ++k) pool.emplace_back(worker);
    worker();
    for (std::thread& th : pool) th.join();
    for (size_t i = 0; i < deferred.size(); ++i) {
      const int64_t base = (int64_t)out.size() - 1;  // local node j >= 1 -> base + j
      auto map = [&](int64_t j) { return j < 0 ? j : base + j; };
      pt_bvh_node& root = out[(size_t)deferred[i].node];
      root.left = map(sub[i][0].left);
      root.right = map(sub[i][0].right);
      for (size_t j = 1; j < sub[i].size(); ++j) {
        pt_bvh_node d = sub[i][j];
        d.left = map(d.left);
        d.right = map(d.right);
        out.push_back(d);
      }
    }
  }
}

}  // namespace

extern "C" int pt_host_build_render_tree(const pt_scene* s, pt_bvh_node* nodes, int64_t* n_nodes, int64_t* perm) {
  if (!s || !nodes || !n_nodes || !perm) return pt_fail(PT_E_INVALID, "pt_host_build_render_tree: NULL argument");
  if (s->n_prims <= 0 || !s->prim_type || !s->prim_geom)
    return pt_fail(PT_E_INVALID, "pt_host_build_render_tree: empty scene");
  for (int64_t i = 0; i < s->n_prims; ++i) {
    if (s->prim_type[i] != PT_PRIM_TRIANGLE && s->prim_type[i] != PT_PRIM_SPHERE)
      return pt_fail(PT_E_INVALID, "pt_host_build_render_tree: unknown primitive type");
    for (int k = 0; k < 9; ++k)
      if (!std::isfinite(s->prim_geom[9 * i + k]))
        return pt_fail(PT_E_INVALID, "pt_host_build_render_tree: non-finite primitive coordinate");
  }
  std::vector<pt_bvh_node> out;
  std::vector<int64_t> pm;
  build_sah_tree(s, out, pm);
  std::memcpy(nodes, out.data(), out.size() * sizeof(pt_bvh_node));
  std::memcpy(perm, pm.data(), pm.size() * sizeof(int64_t));
  *n_nodes = (int64_t)out.size();
  return PT_OK;
}
