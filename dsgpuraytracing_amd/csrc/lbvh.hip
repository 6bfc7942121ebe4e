// lbvh.hip — GPU BVH build (linear BVH) for gfx950.
//
// Replaces the reference's PARALLEL_BUILD_BVH path, CUDAPathTracer::buildBVH
// (cuda_src/setup.cu:478-686) with its kernels computeMorton / generateLeafNode /
// generateInternalNode / buildBoundingBox / treeCollapse (cuda_src/kernel.cu:
// 358-493) and helpers morton3D / delta / determineRange / findSplit /
// propogateBBox (cuda_src/helper.cu:73-91, 354-458):
//   1. 30-bit Morton code of each primitive's box centre in the scene box
//      (the reference's quirks kept: NaN or a coordinate outside [0, 1) -> 0);
//   2. stable key/value radix sort of the codes (thrust::sort_by_key there,
//      hipCUB's onesweep radix sort here);
//   3. Karras 2012 radix tree over (code << 32 | index) keys;
//   4. bottom-up boxes, the second child to arrive completing its parent
//      (agent-scope acquire/release: the per-XCD L2s are not coherent);
//   5. subtrees of <= LEAF_NUMBER = 4 primitives collapse into leaves.
// Beyond the reference (this is the renderer's default tree since round 3):
//   6. treelet restructuring (Karras & Aila 2013): further bottom-up passes
//      (PT_LBVH_PASSES, default 3) rebuild every node's 7-leaf treelet to its
//      SAH optimum by a wave-cooperative dynamic program over the leaf subsets;
//   7. leaves chosen by SAH (a subtree of <= 4 primitives becomes a leaf only
//      where the SAH says a split no longer pays), as the host SAH tree.
// Then, MI355X-specific: the binary tree is emitted both as the 64-B binary
// nodes of the reference-count launch and, breadth-first, as the 128-B BVH4
// nodes the renderer traverses (the largest-area internal child opened until
// four children; children allocated after their parent, so references only
// point forward; primitives numbered in depth-first leaf order); primitives and
// normals are gathered into that order; the worst-case traversal stack is
// computed on the way down.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "pt_device.h"

namespace lbvh {

constexpr int kLeafNumber = 4;  // kernel.cu:14 LEAF_NUMBER

__device__ __forceinline__ uint32_t expand_bits(uint32_t v) {
  v = (v * 0x00010001u) & 0xFF0000FFu;
  v = (v * 0x00000101u) & 0x0F00F00Fu;
  v = (v * 0x00000011u) & 0xC30C30C3u;
  v = (v * 0x00000005u) & 0x49249249u;
  return v;
}

__device__ __forceinline__ uint32_t morton3d(float x, float y, float z) {
  x = fminf(fmaxf(x * 1024.0f, 0.0f), 1023.0f);
  y = fminf(fmaxf(y * 1024.0f, 0.0f), 1023.0f);
  z = fminf(fmaxf(z * 1024.0f, 0.0f), 1023.0f);
  return expand_bits((uint32_t)x) * 4 + expand_bits((uint32_t)y) * 2 + expand_bits((uint32_t)z);
}

// Box of one primitive in the float layout (v0, e1, e2) / (c, r), widened by
// one ulp each way: v0 + e is rounded, the triangle the renderer tests is not.
__device__ __forceinline__ void prim_box(const DPrim& p, float lo[3], float hi[3]) {
  const float v0[3] = {p.v0.x, p.v0.y, p.v0.z};
  if (__float_as_int(p.v0.w) & 1) {
    const float e1[3] = {p.e1.x, p.e1.y, p.e1.z}, e2[3] = {p.e2.x, p.e2.y, p.e2.z};
    for (int i = 0; i < 3; ++i) {
      lo[i] = nextafterf(v0[i] + fminf(fminf(0.0f, e1[i]), e2[i]), -INFINITY);
      hi[i] = nextafterf(v0[i] + fmaxf(fmaxf(0.0f, e1[i]), e2[i]), INFINITY);
    }
  } else {
    for (int i = 0; i < 3; ++i) {
      lo[i] = nextafterf(v0[i] - p.e1.x, -INFINITY);
      hi[i] = nextafterf(v0[i] + p.e1.x, INFINITY);
    }
  }
}

struct Params {
  int n;
  const DPrim* prims;   // input order
  float smin[3], sext[3];
  uint32_t* keys;       // sorted Morton codes
  int* ids;             // sorted primitive ids
  int* child;           // 2 per internal node: >= 0 internal index, < 0: ~leaf (sorted primitive) index
  int* parent;          // parent of internal node i (n-1 entries), then of leaf j (n entries)
  int* start;           // first primitive (final order) of internal node i (written by the emission)
  int* range;           // primitives below internal node i
  float* box;           // 6 per internal node (lo xyz, hi xyz)
  float* cost;          // SAH cost of the subtree of internal node i (unnormalised)
  int* collapsed;       // 1: internal node i becomes one leaf of its <= kMaxLeaf primitives
  int* flag;            // arrivals per internal node (bottom-up passes)
  int* pos;             // final position of sorted primitive j (depth-first leaf order)
  float ci;             // SAH cost of a primitive test (a traversal step costs 1)
  int max_leaf;         // most primitives in one leaf (<= kMaxLeaf)
  float* dpc;           // BVH4 collapse DP (k_dp): 4 per internal node, cost of its subtree in <= i slots
  int8_t* dpk;          // its choices: slots given to the left child, -1 = as with one slot fewer (null: greedy collapse)
};

// Relaxed agent-scope accesses for tree data shared between the climbing
// threads of one bottom-up pass (ordered by the acq_rel arrival counters; the
// XCD L2s are not coherent for plain accesses).
template <class T>
__device__ __forceinline__ T ald(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void ast(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_morton(Params P) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P.n) return;
  const DPrim p = P.prims[i];
  float c[3];
  if (__float_as_int(p.v0.w) & 1) {  // triangle: centre of its box (kernel.cu:366-374)
    const float v0[3] = {p.v0.x, p.v0.y, p.v0.z};
    const float e1[3] = {p.e1.x, p.e1.y, p.e1.z}, e2[3] = {p.e2.x, p.e2.y, p.e2.z};
    for (int k = 0; k < 3; ++k)
      c[k] = v0[k] + 0.5f * (fminf(fminf(0.0f, e1[k]), e2[k]) + fmaxf(fmaxf(0.0f, e1[k]), e2[k]));
  } else {
    c[0] = p.v0.x;
    c[1] = p.v0.y;
    c[2] = p.v0.z;
  }
  for (int k = 0; k < 3; ++k) {
    c[k] = (c[k] - P.smin[k]) / P.sext[k];
    if (c[k] != c[k]) c[k] = 0.0f;
    if (c[k] < 0.0f || c[k] >= 1.0f) c[k] = 0.0f;
  }
  P.keys[i] = morton3d(c[0], c[1], c[2]);
  P.ids[i] = i;
}

__device__ __forceinline__ int delta(const Params& P, int i, int j) {
  if (i < 0 || i >= P.n || j < 0 || j >= P.n) return -1;
  const uint64_t a = ((uint64_t)P.keys[i] << 32) | (uint32_t)i;
  const uint64_t b = ((uint64_t)P.keys[j] << 32) | (uint32_t)j;
  return __clzll((long long)(a ^ b));
}

// Karras 2012: range and split of internal node i (helper.cu:371-435).
__global__ void k_internal(Params P) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P.n - 1) return;
  const int d = (delta(P, i, i + 1) - delta(P, i, i - 1)) >= 0 ? 1 : -1;
  const int dmin = delta(P, i, i - d);
  int lmax = 2;
  while (delta(P, i, i + lmax * d) > dmin) lmax <<= 1;
  int l = 0;
  for (int t = lmax >> 1; t >= 1; t >>= 1)
    if (delta(P, i, i + (l + t) * d) > dmin) l += t;
  const int j = i + l * d;
  const int first = min(i, j), last = max(i, j);
  const int common = delta(P, first, last);
  int split = first, step = last - first;
  do {
    step = (step + 1) >> 1;
    const int ns = split + step;
    if (ns < last && delta(P, first, ns) > common) split = ns;
  } while (step > 1);
  const int a = split == first ? ~split : split;
  const int b = split + 1 == last ? ~(split + 1) : split + 1;
  P.child[2 * i] = a;
  P.child[2 * i + 1] = b;
  P.parent[a >= 0 ? a : (P.n - 1) + ~a] = i;
  P.parent[b >= 0 ? b : (P.n - 1) + ~b] = i;
  P.start[i] = first;
  P.range[i] = last - first + 1;
  P.collapsed[i] = 0;
  P.flag[i] = 0;
  if (i == 0) P.parent[0] = -1;
}

__device__ __forceinline__ void child_box(const Params& P, int c, float lo[3], float hi[3]) {
  if (c < 0) {
    prim_box(P.prims[P.ids[~c]], lo, hi);
  } else {
    for (int k = 0; k < 3; ++k) {
      lo[k] = ald(&P.box[6 * c + k]);
      hi[k] = ald(&P.box[6 * c + 3 + k]);
    }
  }
}

// SAH over the binary tree, as the host render tree (render_tree.cpp): one
// unit per traversal step, one per primitive test, leaves of <= 4 primitives.
constexpr float kCt = 1.0f;
constexpr int kMaxLeaf = 8;  // leaf cursors hold <= 8 primitives; P.max_leaf (default 4) is the SAH's limit
constexpr int kTreelet = 7;  // treelet leaves (Karras & Aila: 7)

__device__ __forceinline__ float half_area(const float lo[3], const float hi[3]) {
  const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
  return dx * dy + dy * dz + dz * dx;
}
__device__ __forceinline__ int node_count(const Params& P, int c) { return c < 0 ? 1 : ald(&P.range[c]); }
__device__ __forceinline__ float node_cost(const Params& P, int c, const float lo[3], const float hi[3]) {
  return c < 0 ? P.ci * half_area(lo, hi) : ald(&P.cost[c]);
}

// Box, count, SAH cost and leaf-collapse choice of internal node `node` from
// its (final) children.
__device__ void node_update(const Params& P, int node, int c0, int c1, int cnt) {
  float la[3], ha[3], lb[3], hb[3], blo[3], bhi[3];
  child_box(P, c0, la, ha);
  child_box(P, c1, lb, hb);
  for (int k = 0; k < 3; ++k) {
    blo[k] = fminf(la[k], lb[k]);
    bhi[k] = fmaxf(ha[k], hb[k]);
    ast(&P.box[6 * node + k], blo[k]);
    ast(&P.box[6 * node + 3 + k], bhi[k]);
  }
  const float a = half_area(blo, bhi);
  const float csplit = kCt * a + node_cost(P, c0, la, ha) + node_cost(P, c1, lb, hb);
  const float cleaf = cnt <= P.max_leaf ? P.ci * a * (float)cnt : INFINITY;
  ast(&P.range[node], cnt);
  ast(&P.cost[node], fminf(csplit, cleaf));
  ast(&P.collapsed[node], cleaf <= csplit ? 1 : 0);
}

// SAH-optimal rebuild of the treelet rooted at R (wave-uniform), by the whole
// wave: the treelet is R's kTreelet largest-area descendants (leaves); the DP
// over the leaf subsets runs one subset size at a time, the subsets of one
// size on parallel lanes, each lane scanning its subset's partitions; lane 0
// then rewrites the treelet's internal nodes from the DP choices.
__device__ void treelet_wave(const Params& P, int R, int lane, float* s_cost, uint8_t* s_pick, uint8_t* s_coll) {
  int leaf[kTreelet], inner[kTreelet - 1];
  float lo[kTreelet][3], hi[kTreelet][3];
  int nl = 2, ni = 1;
  leaf[0] = ald(&P.child[2 * R]);
  leaf[1] = ald(&P.child[2 * R + 1]);
  inner[0] = R;
  child_box(P, leaf[0], lo[0], hi[0]);
  child_box(P, leaf[1], lo[1], hi[1]);
  while (nl < kTreelet) {
    int best = -1;
    float ba = -1.0f;
    for (int i = 0; i < nl; ++i)
      if (leaf[i] >= 0) {
        const float a = half_area(lo[i], hi[i]);
        if (a > ba) {
          ba = a;
          best = i;
        }
      }
    if (best < 0) break;
    const int x = leaf[best];
    inner[ni++] = x;
    leaf[best] = ald(&P.child[2 * x]);
    leaf[nl] = ald(&P.child[2 * x + 1]);
    child_box(P, leaf[best], lo[best], hi[best]);
    child_box(P, leaf[nl], lo[nl], hi[nl]);
    ++nl;
  }
  float lcost[kTreelet];
  int lcnt[kTreelet];
  for (int i = 0; i < nl; ++i) {
    lcost[i] = node_cost(P, leaf[i], lo[i], hi[i]);
    lcnt[i] = node_count(P, leaf[i]);
  }
  const int full = (1 << nl) - 1;
  if (lane < nl) s_cost[1 << lane] = lcost[lane];
  __syncthreads();
  for (int k = 2; k <= nl; ++k) {
    for (int S = lane + 1; S <= full; S += 64) {
      if (__popc(S) != k) continue;
      float blo[3] = {INFINITY, INFINITY, INFINITY}, bhi[3] = {-INFINITY, -INFINITY, -INFINITY};
      int n = 0;
      for (int i = 0; i < nl; ++i)
        if (S & (1 << i)) {
          n += lcnt[i];
          for (int q = 0; q < 3; ++q) {
            blo[q] = fminf(blo[q], lo[i][q]);
            bhi[q] = fmaxf(bhi[q], hi[i][q]);
          }
        }
      const float a = half_area(blo, bhi);
      // partitions (P, S \ P) with P holding S's lowest leaf: each once
      const int low = S & -S, rest = S ^ low;
      float best = INFINITY;
      int bp = low;
      for (int sub = (rest - 1) & rest;; sub = (sub - 1) & rest) {
        const int Pm = low | sub;
        const float c = s_cost[Pm] + s_cost[S ^ Pm];
        if (c < best) {
          best = c;
          bp = Pm;
        }
        if (sub == 0) break;
      }
      const float csplit = kCt * a + best;
      const float cleaf = n <= P.max_leaf ? P.ci * a * (float)n : INFINITY;
      s_pick[S] = (uint8_t)bp;
      s_coll[S] = cleaf <= csplit ? 1 : 0;
      s_cost[S] = fminf(csplit, cleaf);
    }
    __syncthreads();
  }
  if (lane == 0) {
    // rebuild top-down, reusing the treelet's internal nodes (the root keeps
    // its index and its parent)
    int stk_s[kTreelet], stk_x[kTreelet], sp = 0, next = 1;
    stk_s[sp] = full;
    stk_x[sp++] = R;
    while (sp > 0) {
      --sp;
      const int S = stk_s[sp], x = stk_x[sp];
      const int parts[2] = {s_pick[S], S ^ s_pick[S]};
      for (int side = 0; side < 2; ++side) {
        const int sub = parts[side];
        int c;
        if ((sub & (sub - 1)) == 0) {
          c = leaf[__ffs(sub) - 1];
        } else {
          c = inner[next++];
          stk_s[sp] = sub;
          stk_x[sp++] = c;
        }
        ast(&P.child[2 * x + side], c);
        ast(&P.parent[c >= 0 ? c : (P.n - 1) + ~c], x);
      }
      float blo[3] = {INFINITY, INFINITY, INFINITY}, bhi[3] = {-INFINITY, -INFINITY, -INFINITY};
      int n = 0;
      for (int i = 0; i < nl; ++i)
        if (S & (1 << i)) {
          n += lcnt[i];
          for (int q = 0; q < 3; ++q) {
            blo[q] = fminf(blo[q], lo[i][q]);
            bhi[q] = fmaxf(bhi[q], hi[i][q]);
          }
        }
      for (int q = 0; q < 3; ++q) {
        ast(&P.box[6 * x + q], blo[q]);
        ast(&P.box[6 * x + 3 + q], bhi[q]);
      }
      ast(&P.range[x], n);
      ast(&P.cost[x], s_cost[S]);
      ast(&P.collapsed[x], (int)s_coll[S]);
    }
  }
  __syncthreads();  // the tables are reused by the wave's next treelet
}

// Bottom-up pass (propogateBBox, helper.cu:437-458, extended): one lane per
// primitive climbs until it is the first to reach a node; the second arrival
// owns the node, whose children are final, and sets its box, count, SAH cost
// and leaf-collapse choice -- with `optimize`, for nodes with >= kTreelet
// primitives, after the wave has rebuilt the node's treelet.  Lanes stay in
// the loop (idle) until every lane of the wave has finished climbing, so the
// whole wave takes part in every treelet's DP.  One wave per workgroup.
__global__ __launch_bounds__(64) void k_treelet(Params P, int optimize) {
  __shared__ float s_cost[128];
  __shared__ uint8_t s_pick[128], s_coll[128];
  const int lane = threadIdx.x;
  const int j = blockIdx.x * 64 + lane;
  bool active = j < P.n && P.n >= 2;
  int node = active ? ald(&P.parent[(P.n - 1) + j]) : -1;
  for (;;) {
    if (active) {
      if (node < 0) active = false;
      else if (__hip_atomic_fetch_add(&P.flag[node], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == 0)
        active = false;  // the first arrival: the sibling subtree is not finished
    }
    if (__ballot(active) == 0ull) break;
    int c0 = 0, c1 = 0, cnt = 0;
    if (active) {
      c0 = ald(&P.child[2 * node]);
      c1 = ald(&P.child[2 * node + 1]);
      cnt = node_count(P, c0) + node_count(P, c1);
    }
    const bool opt = active && optimize && cnt >= kTreelet;
    unsigned long long m = __ballot(opt);
    while (m != 0ull) {
      const int l = __ffsll((long long)m) - 1;
      m &= m - 1ull;
      treelet_wave(P, __shfl(node, l), lane, s_cost, s_pick, s_coll);
    }
    if (active && !opt) node_update(P, node, c0, c1, cnt);
    if (active) node = ald(&P.parent[node]);
  }
}

// ---- SAH-optimal BVH4 collapse (round 5): dynamic programming over (binary
// node, slots), Ylitie et al. 2017's wide-BVH DP at width 4.  D(n, i) is the
// least expected cost of n's subtree when it fills at most i slots of its
// parent BVH4 node, in the kernel's units: a node step or a leaf step (two
// primitives) costs one, weighted by surface area.  Leaves (primitives and
// collapsed subtrees) fill one slot; an internal node kept whole costs
// A(n) + the best split of its two children over four slots; with i >= 2
// slots it may also be opened, its children sharing the i slots.  The greedy
// collapse (open the largest-area child until four) leaves many nodes with two
// or three children; on the C3 ray mix the DP tree takes 6-13% fewer steps per
// ray (tools/wide_sim.cpp).
__device__ __forceinline__ float dp_cost(const Params& P, int c, int i) {
  if (c < 0) {
    float lo[3], hi[3];
    prim_box(P.prims[P.ids[~c]], lo, hi);
    return half_area(lo, hi);
  }
  if (ald(&P.collapsed[c])) {
    float lo[3], hi[3];
    child_box(P, c, lo, hi);
    return half_area(lo, hi) * (float)((ald(&P.range[c]) + 1) / 2);
  }
  return ald(&P.dpc[4 * c + (i - 1)]);
}

__device__ void dp_update(const Params& P, int n) {
  const int c0 = ald(&P.child[2 * n]), c1 = ald(&P.child[2 * n + 1]);
  float a0[5], a1[5];
  for (int i = 1; i <= 4; ++i) {
    a0[i] = dp_cost(P, c0, i);
    a1[i] = dp_cost(P, c1, i);
  }
  float dist[5];
  int8_t arg[5];
  for (int j = 2; j <= 4; ++j) {
    dist[j] = INFINITY;
    arg[j] = 1;
    for (int k = 1; k < j; ++k) {
      const float c = a0[k] + a1[j - k];
      if (c < dist[j]) {
        dist[j] = c;
        arg[j] = (int8_t)k;
      }
    }
  }
  float lo[3], hi[3];
  child_box(P, n, lo, hi);
  float prev = kCt * half_area(lo, hi) + dist[4];
  ast(&P.dpc[4 * n], prev);
  ast(&P.dpk[4 * n], arg[4]);  // (for i = 1: the split of the node kept whole)
  for (int i = 2; i <= 4; ++i) {
    const bool open = dist[i] < prev;
    prev = open ? dist[i] : prev;
    ast(&P.dpc[4 * n + (i - 1)], prev);
    ast(&P.dpk[4 * n + (i - 1)], open ? arg[i] : (int8_t)-1);
  }
}

// Bottom-up DP pass: one lane per primitive climbs; the second arrival at a
// node owns it (its children's tables are final).  P.flag must be zero.
__global__ void k_dp(Params P) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= P.n || P.n < 2) return;
  int node = ald(&P.parent[(P.n - 1) + j]);
  while (node >= 0) {
    if (__hip_atomic_fetch_add(&P.flag[node], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
    dp_update(P, node);
    node = ald(&P.parent[node]);
  }
}

struct Item {
  int bin;    // internal binary node (not collapsed)
  int idx;    // its BVH4 node index
  int stack;  // worst-case stack entries on entering it
  int start;  // its first primitive in the final (depth-first leaf) order
};

__device__ __forceinline__ int cursor(int first, int count) { return ~((first << 3) | (count - 1)); }

// One BVH4 node per item, top-down: open the largest-area internal child
// (not collapsed) until four children; every child gets its first primitive
// in depth-first leaf order, collapsed subtrees and primitives become leaf
// cursors (their primitives numbered here), internal children are queued
// with a freshly allocated (forward) index.
__global__ void k_bfs(Params P, const Item* __restrict__ in, int n_in, Item* out, int* n_out, int* n_nodes,
                      int* max_stack, DNode* nodes) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_in) return;
  const Item it = in[t];
  P.start[it.bin] = it.start;
  int kids[4], ks[4];
  float klo[4][3], khi[4][3];
  int nk = 2;
  if (P.dpk) {
    // the DP's choice: the node's two children over four slots, each opened
    // as its table says; children in depth-first (left to right) order
    int sx[8], si[8], sp = 0;
    const int k4 = P.dpk[4 * it.bin];
    sx[sp] = P.child[2 * it.bin + 1];
    si[sp++] = 4 - k4;
    sx[sp] = P.child[2 * it.bin];
    si[sp++] = k4;
    nk = 0;
    while (sp > 0) {
      --sp;
      const int x = sx[sp];
      int i = si[sp];
      if (x >= 0 && !P.collapsed[x]) {
        while (i > 1 && P.dpk[4 * x + (i - 1)] == -1) --i;
        if (i > 1) {
          const int k = P.dpk[4 * x + (i - 1)];
          sx[sp] = P.child[2 * x + 1];
          si[sp++] = i - k;
          sx[sp] = P.child[2 * x];
          si[sp++] = k;
          continue;
        }
      }
      kids[nk++] = x;
    }
    ks[0] = it.start;
    for (int k = 0; k < nk; ++k) {
      if (k > 0) ks[k] = ks[k - 1] + node_count(P, kids[k - 1]);
      child_box(P, kids[k], klo[k], khi[k]);
    }
  } else {
  kids[0] = P.child[2 * it.bin];
  kids[1] = P.child[2 * it.bin + 1];
  ks[0] = it.start;
  ks[1] = it.start + node_count(P, kids[0]);
  child_box(P, kids[0], klo[0], khi[0]);
  child_box(P, kids[1], klo[1], khi[1]);
  while (nk < 4) {
    int best = -1;
    float ba = -1.0f;
    for (int k = 0; k < nk; ++k)
      if (kids[k] >= 0 && !P.collapsed[kids[k]]) {
        const float a = half_area(klo[k], khi[k]);
        if (a > ba) {
          ba = a;
          best = k;
        }
      }
    if (best < 0) break;
    const int x = kids[best];
    P.start[x] = ks[best];
    kids[best] = P.child[2 * x];
    kids[nk] = P.child[2 * x + 1];
    ks[nk] = ks[best] + node_count(P, kids[best]);
    child_box(P, kids[best], klo[best], khi[best]);
    child_box(P, kids[nk], klo[nk], khi[nk]);
    ++nk;
  }
  }
  const int below = it.stack + nk - 1;
  atomicMax(max_stack, below);
  float lo[3][4], hi[3][4];
  int ref[4];
  for (int k = 0; k < 4; ++k) {
    if (k < nk) {
      for (int a = 0; a < 3; ++a) {
        lo[a][k] = klo[k][a];
        hi[a][k] = khi[k][a];
      }
      const int c = kids[k];
      int r;
      if (c < 0) {  // one primitive
        P.pos[~c] = ks[k];
        r = cursor(ks[k], 1);
      } else if (P.collapsed[c]) {  // a leaf of its <= kMaxLeaf primitives, numbered depth-first
        P.start[c] = ks[k];
        int st[kMaxLeaf + 1], sp = 0, m = ks[k];  // depth-first, left child first
        st[sp++] = c;
        while (sp > 0) {
          const int x = st[--sp];
          if (x < 0) {
            P.pos[~x] = m++;
          } else {
            st[sp++] = P.child[2 * x + 1];
            st[sp++] = P.child[2 * x];
          }
        }
        r = cursor(ks[k], P.range[c]);
      } else {
        const int idx = atomicAdd(n_nodes, 1);
        out[atomicAdd(n_out, 1)] = Item{c, idx, below, ks[k]};
        r = idx;
      }
      ref[k] = r;
    } else {  // empty slot: box at +inf, a leaf cursor (never entered)
      for (int a = 0; a < 3; ++a) lo[a][k] = hi[a][k] = __int_as_float(0x7f800000);
      ref[k] = cursor(0, 1);
    }
  }
  DNode d;
  d.lox = make_float4(lo[0][0], lo[0][1], lo[0][2], lo[0][3]);
  d.hix = make_float4(hi[0][0], hi[0][1], hi[0][2], hi[0][3]);
  d.loy = make_float4(lo[1][0], lo[1][1], lo[1][2], lo[1][3]);
  d.hiy = make_float4(hi[1][0], hi[1][1], hi[1][2], hi[1][3]);
  d.loz = make_float4(lo[2][0], lo[2][1], lo[2][2], lo[2][3]);
  d.hiz = make_float4(hi[2][0], hi[2][1], hi[2][2], hi[2][3]);
  d.ref = make_int4(ref[0], ref[1], ref[2], ref[3]);
  d.pad = make_int4(0, 0, 0, 0);
  nodes[it.idx] = d;
}

// Binary nodes for the reference-count launch (node index = Karras index),
// children as the renderer sees them: primitives and collapsed subtrees are
// leaf cursors over the final order, other internal nodes their index.
__device__ __forceinline__ int as_ref(const Params& P, int c) {
  if (c < 0) return cursor(P.pos[~c], 1);
  if (P.collapsed[c]) return cursor(P.start[c], P.range[c]);
  return c;
}

__global__ void k_emit_bin(Params P, DNode2* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P.n - 1) return;
  float l0[3], h0[3], l1[3], h1[3];
  const int c0 = P.child[2 * i], c1 = P.child[2 * i + 1];
  child_box(P, c0, l0, h0);
  child_box(P, c1, l1, h1);
  DNode2 d;
  d.a = make_float4(l0[0], h0[0], l0[1], h0[1]);
  d.b = make_float4(l1[0], h1[0], l1[1], h1[1]);
  d.c = make_float4(l0[2], h0[2], l1[2], h1[2]);
  d.e = make_int4(as_ref(P, c0), as_ref(P, c1), 0, 0);
  out[i] = d;
}

__global__ void k_identity(Params P) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < P.n) P.pos[j] = j;
}

// Primitives, vertex normals and the final -> input id map in the final
// (depth-first leaf) order.
__global__ void k_gather(Params P, const float* __restrict__ norms_in, DPrim* prims_out, float* norms_out,
                         int* prim_map) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= P.n) return;
  const int s = P.ids[j];
  const int i = P.pos[j];
  prims_out[i] = P.prims[s];
  for (int k = 0; k < 9; ++k) norms_out[9 * (size_t)i + k] = norms_in[9 * (size_t)s + k];
  prim_map[i] = s;
}

}  // namespace lbvh

#define LB_CHK(x)                   \
  do {                              \
    hipError_t e_ = (x);            \
    if (e_ != hipSuccess) return e_; \
  } while (0)

extern "C" hipError_t ptk_build_lbvh(const LbvhIn* in, LbvhOut* out, hipStream_t s) {
  using namespace lbvh;
  const int n = in->n;
  *out = LbvhOut{};
  Params P{};
  P.n = n;
  P.prims = in->prims;
  for (int k = 0; k < 3; ++k) {
    P.smin[k] = in->scene_min[k];
    P.sext[k] = in->scene_extent[k];
  }
  int passes = 3;  // treelet-restructuring passes (0: the reference's Karras tree, SAH leaf collapse)
  if (const char* e = std::getenv("PT_LBVH_PASSES")) passes = std::max(0, std::min(8, std::atoi(e)));
  P.ci = 1.0f;      // the host SAH tree's costs (render_tree.cpp)
  P.max_leaf = 4;
  if (const char* e = std::getenv("PT_LBVH_CI")) P.ci = std::max(0.05f, std::min(8.0f, (float)std::atof(e)));  // tuning knobs
  if (const char* e = std::getenv("PT_LBVH_MAXLEAF")) P.max_leaf = std::max(1, std::min(kMaxLeaf, std::atoi(e)));
  // scratch
  uint32_t *keys_a = nullptr, *keys_b = nullptr;
  int *ids_a = nullptr, *ids_b = nullptr, *ints = nullptr;
  float *box = nullptr, *cost = nullptr, *dpc = nullptr;
  int8_t* dpk = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  const size_t ni = (size_t)(n > 1 ? n - 1 : 1);
  LB_CHK(hipMalloc(&keys_a, (size_t)n * 4));
  LB_CHK(hipMalloc(&keys_b, (size_t)n * 4));
  LB_CHK(hipMalloc(&ids_a, (size_t)n * 4));
  LB_CHK(hipMalloc(&ids_b, (size_t)n * 4));
  // child 2ni, parent ni+n, start ni, range ni, collapsed ni, flag ni, pos n, counters 4
  LB_CHK(hipMalloc(&ints, (ni * 2 + (ni + n) + ni * 4 + n + 4) * 4));
  LB_CHK(hipMalloc(&box, ni * 6 * 4));
  LB_CHK(hipMalloc(&cost, ni * 4));
  const int B = 256;
  const int gn = (n + B - 1) / B, gi = (int)((ni + B - 1) / B);
  P.keys = keys_a;
  P.ids = ids_a;
  hipLaunchKernelGGL(k_morton, dim3(gn), dim3(B), 0, s, P);
  LB_CHK(hipGetLastError());
  LB_CHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, keys_a, keys_b, ids_a, ids_b, n, 0, 30, s));
  LB_CHK(hipMalloc(&tmp, tmp_bytes));
  LB_CHK(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys_a, keys_b, ids_a, ids_b, n, 0, 30, s));
  P.keys = keys_b;
  P.ids = ids_b;
  P.child = ints;
  P.parent = P.child + 2 * ni;
  P.start = P.parent + ni + n;
  P.range = P.start + ni;
  P.collapsed = P.range + ni;
  P.flag = P.collapsed + ni;
  P.pos = P.flag + ni;
  int* counters = P.pos + n;  // n_nodes, n_out, max_stack, spare
  P.box = box;
  P.cost = cost;
  LB_CHK(hipMemsetAsync(counters, 0, 16, s));
  // outputs
  LB_CHK(hipMalloc(&out->prims, (size_t)n * sizeof(DPrim)));
  LB_CHK(hipMalloc(&out->norms, (size_t)n * 9 * 4));
  LB_CHK(hipMalloc(&out->prim_map, (size_t)n * 4));
  LB_CHK(hipMalloc(&out->nodes4, (size_t)(ni + 1) * sizeof(DNode)));
  LB_CHK(hipMalloc(&out->nodes2, ni * sizeof(DNode2)));
  if (n <= kLeafNumber) {  // a single leaf: one BVH4 node, one child, as the host path
    hipLaunchKernelGGL(k_identity, dim3(gn), dim3(B), 0, s, P);  // final order = sorted order
    LB_CHK(hipGetLastError());
    hipLaunchKernelGGL(k_gather, dim3(gn), dim3(B), 0, s, P, in->norms, out->prims, out->norms, out->prim_map);
    LB_CHK(hipGetLastError());
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int k = 0; k < 3; ++k) {
      lo[k] = in->scene_min[k];
      hi[k] = in->scene_min[k] + in->scene_extent[k];
    }
    DNode d{};
    float inf = INFINITY;
    d.lox = make_float4(lo[0], inf, inf, inf);
    d.hix = make_float4(hi[0], inf, inf, inf);
    d.loy = make_float4(lo[1], inf, inf, inf);
    d.hiy = make_float4(hi[1], inf, inf, inf);
    d.loz = make_float4(lo[2], inf, inf, inf);
    d.hiz = make_float4(hi[2], inf, inf, inf);
    d.ref = make_int4(~((0 << 3) | (n - 1)), ~0, ~0, ~0);
    LB_CHK(hipMemcpyAsync(out->nodes4, &d, sizeof(d), hipMemcpyHostToDevice, s));
    DNode2 b{};
    b.a = make_float4(lo[0], hi[0], lo[1], hi[1]);
    b.b = make_float4(inf, inf, inf, inf);
    b.c = make_float4(lo[2], hi[2], inf, inf);
    b.e = make_int4(~((0 << 3) | (n - 1)), ~0, 0, 0);
    LB_CHK(hipMemcpyAsync(out->nodes2, &b, sizeof(b), hipMemcpyHostToDevice, s));
    LB_CHK(hipStreamSynchronize(s));
    out->n4 = 1;
    out->n2 = 1;
    out->max_stack = 1;
    for (int k = 0; k < 3; ++k) {
      out->root_lo[k] = lo[k];
      out->root_hi[k] = hi[k];
    }
  } else {
    hipLaunchKernelGGL(k_internal, dim3(gi), dim3(B), 0, s, P);
    LB_CHK(hipGetLastError());
    // bottom-up: boxes, counts, SAH costs, leaf collapse; then the treelet passes
    // (the first pass sets every node's box and cost on its way up too)
    const int gt = (n + 63) / 64;
    for (int p = 0; p < std::max(1, passes); ++p) {
      if (p > 0) LB_CHK(hipMemsetAsync(P.flag, 0, ni * 4, s));
      hipLaunchKernelGGL(k_treelet, dim3(gt), dim3(64), 0, s, P, passes > 0 ? 1 : 0);
      LB_CHK(hipGetLastError());
    }
    // the BVH4 collapse: greedy (default: open the largest-area child until
    // four) or the SAH-optimal DP (PT_COLLAPSE=dp).  Over this tree the DP
    // changes little -- C3 traversal steps -0.6%, throughput +-0.2%, C4
    // +0.7%, C5 / c5big -1.5% (profiles/r5/ab_collapse_dp.txt): the treelet
    // passes already leave a tree whose greedy collapse is near the SAH
    // optimum; over the host SAH tree it pays (+10%, pt_api.cpp).
    const char* ce = std::getenv("PT_COLLAPSE");
    if (ce && std::strcmp(ce, "dp") == 0) {
      LB_CHK(hipMalloc(&dpc, ni * 4 * sizeof(float)));
      LB_CHK(hipMalloc(&dpk, ni * 4));
      P.dpc = dpc;
      P.dpk = dpk;
      LB_CHK(hipMemsetAsync(P.flag, 0, ni * 4, s));
      hipLaunchKernelGGL(k_dp, dim3(gn), dim3(B), 0, s, P);
      LB_CHK(hipGetLastError());
    }
    // top-down BVH4 emission (breadth first, binary node 0 -> BVH4 node 0),
    // numbering the primitives in depth-first leaf order on the way
    Item *fa = nullptr, *fb = nullptr;
    LB_CHK(hipMalloc(&fa, (ni + 1) * sizeof(Item)));
    LB_CHK(hipMalloc(&fb, (ni + 1) * sizeof(Item)));
    Item root{0, 0, 0, 0};
    int one = 1;
    LB_CHK(hipMemcpyAsync(fa, &root, sizeof(root), hipMemcpyHostToDevice, s));
    LB_CHK(hipMemcpyAsync(counters, &one, 4, hipMemcpyHostToDevice, s));  // n_nodes = 1 (the root)
    int n_in = 1;
    while (n_in > 0) {  // one launch per BVH4 level
      LB_CHK(hipMemsetAsync(counters + 1, 0, 4, s));
      hipLaunchKernelGGL(k_bfs, dim3((n_in + B - 1) / B), dim3(B), 0, s, P, fa, n_in, fb, counters + 1, counters,
                         counters + 2, out->nodes4);
      LB_CHK(hipGetLastError());
      LB_CHK(hipMemcpyAsync(&n_in, counters + 1, 4, hipMemcpyDeviceToHost, s));
      LB_CHK(hipStreamSynchronize(s));
      Item* t = fa;
      fa = fb;
      fb = t;
    }
    hipLaunchKernelGGL(k_emit_bin, dim3(gi), dim3(B), 0, s, P, out->nodes2);
    LB_CHK(hipGetLastError());
    hipLaunchKernelGGL(k_gather, dim3(gn), dim3(B), 0, s, P, in->norms, out->prims, out->norms, out->prim_map);
    LB_CHK(hipGetLastError());
    int cnt[3] = {0, 0, 0};
    LB_CHK(hipMemcpyAsync(cnt, counters, 12, hipMemcpyDeviceToHost, s));
    float rb[6];
    LB_CHK(hipMemcpyAsync(rb, box, 24, hipMemcpyDeviceToHost, s));
    LB_CHK(hipStreamSynchronize(s));
    out->n4 = cnt[0];
    out->n2 = (int)ni;
    out->max_stack = cnt[2];
    for (int k = 0; k < 3; ++k) {
      out->root_lo[k] = rb[k];
      out->root_hi[k] = rb[3 + k];
    }
    (void)hipFree(fa);
    (void)hipFree(fb);
  }
  (void)hipFree(keys_a);
  (void)hipFree(keys_b);
  (void)hipFree(ids_a);
  (void)hipFree(ids_b);
  (void)hipFree(ints);
  (void)hipFree(box);
  if (dpc) (void)hipFree(dpc);
  if (dpk) (void)hipFree(dpk);
  (void)hipFree(cost);
  (void)hipFree(tmp);
  return hipSuccess;
}
