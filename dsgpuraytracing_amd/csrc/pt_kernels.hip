// pt_kernels.hip — gfx950 (CDNA4) kernels of the path-tracing hot path.
//
// Replaces the reference's per-pixel radiance loop:
//   CPU: PathTracer::raytrace_tile -> raytrace_pixel -> trace_ray
//        (src/pathtracer.cpp:407-611) over BVHAccel (src/bvh.cpp:227-362)
//   GPU: traceScenePT -> tracePixelPT -> traceRay (cuda_src/kernel.cu:31-349),
//        BVH_traversal (traversal.cu:3-222), intersect.cu, bsdf.cu, light.cu
//
// Design (MI355X-first, not a translation):
//  * one persistent megakernel, one wave64 per workgroup; a lane owns one
//    (pixel, sample group) work slot at a time, renders its samples in order
//    and stores their sum; resolve_kernel sums a pixel's groups in a fixed order
//    (deterministic, no float atomics, independent of tile->GPU assignment);
//  * the recursion of trace_ray becomes an iterative throughput loop driven by a
//    per-lane state machine that owns exactly ONE ray (extension or shadow);
//    rounds alternate a shading phase (finished lanes shade and refill from a
//    wave-chunked atomic queue over footprint-clipped 8x8 pixel blocks) and a
//    traversal phase that runs until shade_batch lanes are done;
//  * if-if traversal: each iteration the wave runs either node steps (BVH4,
//    128-B SoA node, 4 slab tests, sorting-network near-first order) or leaf
//    steps (two primitives per step, loads issued together), whichever kind
//    more lanes wait on; leaves are cursors in the child references;
//  * traversal stack per lane in LDS (lane-contiguous, conflict-free);
//    material/light tables staged in LDS;
//  * fp32 throughout; self-intersection handled by the integer-ulp origin offset
//    (Waechter & Binder, Ray Tracing Gems ch.6) instead of the reference's
//    EPS_D = 1e-11 double offsets, which are meaningless in fp32.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

#include "pt_device.h"
#include "pt_rng.h"

#ifndef PT_ENV_TU
#define PT_ENV_TU 0
#endif

namespace ptk {

__device__ __forceinline__ float3 f3(float x, float y, float z) { return make_float3(x, y, z); }
__device__ __forceinline__ float3 operator+(float3 a, float3 b) { return f3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ float3 operator-(float3 a, float3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ float3 operator*(float3 a, float s) { return f3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ float3 operator*(float s, float3 a) { return f3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ float3 mul(float3 a, float3 b) { return f3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ float dot(float3 a, float3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float3 cross(float3 u, float3 v) {
  return f3(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
// v_rsq_f32 / v_rcp_f32 (about 1 ulp): the shading frame and the triangle
// determinant do not need IEEE division's last bit, and one instruction
// replaces a ~10-instruction correctly rounded sequence.
__device__ __forceinline__ float3 normalize(float3 v) { return v * __builtin_amdgcn_rsqf(dot(v, v)); }
__device__ __forceinline__ float rcp(float x) { return __builtin_amdgcn_rcpf(x); }
// v_sqrt_f32 (about 1 ulp) for sampling; the sphere test keeps sqrtf
__device__ __forceinline__ float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
// sin / cos of 2*pi*x for x in [0, 1) (v_sin_f32 / v_cos_f32 take revolutions)
__device__ __forceinline__ float sin_rev(float x) { return __builtin_amdgcn_sinf(x); }
__device__ __forceinline__ float cos_rev(float x) { return __builtin_amdgcn_cosf(x); }

// Conservative slab-test factor on the far distance (Ize 2013: 1 + 2*gamma_3
// for exact reciprocals), with margin for the ~1-ulp v_rcp_f32 of 1/d.
#define PT_ROBUST 1.0000008f
__device__ __forceinline__ float illum(float3 s) { return 0.2126f * s.x + 0.7152f * s.y + 0.0722f * s.z; }
// (T: float in any address space -- the launch parameters are read from the
// kernel-argument segment, address space 4)
template <class T>
__device__ __forceinline__ float3 ld3(const T* p) { return f3(p[0], p[1], p[2]); }
__device__ __forceinline__ void store3(float* p, float3 v) {
  p[0] = v.x;
  p[1] = v.y;
  p[2] = v.z;
}
// A group sum (12 B): written once, read once by the resolve.  (Measured and
// removed: non-temporal stores, which trade FETCH_SIZE for WRITE_SIZE at
// throughput within noise -- profiles/r4/ab_nt_sums.txt, r5/ab_nt_sums_final.txt;
// 16-B records, C3 -1.5% -- r5/ab_order_ballot.txt.)
__device__ __forceinline__ void store_sum(float* p, float3 v) { store3(p, v); }
// Pixel q (0..1023) of a tile in 8x8 blocks (4 blocks per row); (-1,-1) when
// it lies outside a ragged tile.
__device__ __forceinline__ int2 tile_pixel(int4 tile, uint32_t q) {
  uint32_t blk = q >> 6, w = q & 63u;
  int x = tile.x + (int)((blk & 3u) * 8u + (w & 7u));
  int y = tile.y + (int)((blk >> 2) * 8u + (w >> 3));
  if (x >= tile.x + tile.z || y >= tile.y + tile.w) return make_int2(-1, -1);
  return make_int2(x, y);
}

// The pixel lies outside the scene box's conservative screen footprint.
__device__ __forceinline__ bool culled(const KParams& P, int x, int y) {
  return x < P.cull_x0 || x > P.cull_x1 || y < P.cull_y0 || y > P.cull_y1;
}

// Integer-ulp offset of p along n (n points to the side the new ray leaves on).
__device__ __forceinline__ float3 offset_ray(float3 p, float3 n) {
  const float kOrigin = 1.0f / 32.0f, kFloatScale = 1.0f / 65536.0f, kIntScale = 256.0f;
  int ox = (int)(kIntScale * n.x), oy = (int)(kIntScale * n.y), oz = (int)(kIntScale * n.z);
  float pix = __int_as_float(__float_as_int(p.x) + (p.x < 0 ? -ox : ox));
  float piy = __int_as_float(__float_as_int(p.y) + (p.y < 0 ? -oy : oy));
  float piz = __int_as_float(__float_as_int(p.z) + (p.z < 0 ? -oz : oz));
  return f3(fabsf(p.x) < kOrigin ? p.x + kFloatScale * n.x : pix,
            fabsf(p.y) < kOrigin ? p.y + kFloatScale * n.y : piy,
            fabsf(p.z) < kOrigin ? p.z + kFloatScale * n.z : piz);
}

// Orthonormal frame as make_coord_space (src/bsdf.cpp:13-30): z = n, and the
// smallest-magnitude component of n replaced by 1 seeds the cross products.
struct Frame {
  float3 x, y, z;
  __device__ __forceinline__ float3 to_local(float3 v) const { return f3(dot(v, x), dot(v, y), dot(v, z)); }
  __device__ __forceinline__ float3 to_world(float3 v) const { return x * v.x + y * v.y + z * v.z; }
};
__device__ __forceinline__ Frame make_frame(float3 n) {
  Frame f;
  float3 z = normalize(n);
  float3 h = n;
  float ax = fabsf(h.x), ay = fabsf(h.y), az = fabsf(h.z);
  if (ax <= ay && ax <= az) h.x = 1.0f;
  else if (ay <= ax && ay <= az) h.y = 1.0f;
  else h.z = 1.0f;
  float3 y = normalize(cross(h, z));
  f.x = normalize(cross(z, y));
  f.y = y;
  f.z = z;
  return f;
}

// Materialises loaded values in VGPRs at this point (an empty asm that
// "modifies" them): the loads must be issued before it and cannot be sunk
// into later branches (node steps, leaf steps and the hit record).
#define PT_FENCE4(v) asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w))
#define PT_FENCE3(v) asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z))

struct RayState {
  float3 o, d;
  float tmax;
};

struct Hit {
  float t;
  int prim;
};

struct Counters {
  uint32_t nodes, tris, spheres;
};

// Resumable stack-based BVH2 traversal state of one lane.
// The closest hit is (tmax, prim): the shading round rebuilds the barycentrics
// and reads the material from the primitive record, so no more of the hit is
// carried through traversal (every persistent value costs a VGPR in all waves).
// (Re-deriving the direction from 1/d instead of keeping it measured C3 -1.1%,
// C5 -2.1%: profiles/r5/ab_dfree_*.txt.)
struct Trav {
  float3 o, d, inv;
  float tmax;
  int node, sp;
  int prim;
  bool any, found;
};
__device__ __forceinline__ float3 tdir(const Trav& t) { return t.d; }

__device__ __forceinline__ void trav_init(Trav& tr, float3 o, float3 d, float tmax, bool any) {
  const float kTiny = 1e-20f;
  float3 dd = f3(fabsf(d.x) < kTiny ? copysignf(kTiny, d.x) : d.x, fabsf(d.y) < kTiny ? copysignf(kTiny, d.y) : d.y,
                 fabsf(d.z) < kTiny ? copysignf(kTiny, d.z) : d.z);
  tr.o = o;
  tr.d = d;
  tr.inv = f3(rcp(dd.x), rcp(dd.y), rcp(dd.z));
  tr.tmax = tmax;
  tr.node = 0;
  tr.sp = 0;
  tr.any = any;
  tr.found = false;
  tr.prim = -1;
}

// Moller-Trumbore terms of one triangle (u, v, t; det = 0 means parallel).
// Shared by the traversal test and the shading round's barycentric rebuild,
// which must agree bit for bit.
__device__ __forceinline__ float mt_terms(float3 o, float3 d, float3 V0, float3 E1, float3 E2, float& u, float& v,
                                          float& t) {
  float3 pv = cross(d, E2);
  float det = dot(E1, pv);
  float id = __builtin_amdgcn_rcpf(det);
  float3 tv = o - V0;
  u = dot(tv, pv) * id;
  float3 qv = cross(tv, E1);
  v = dot(d, qv) * id;
  t = dot(E2, qv) * id;
  return det;
}

// Intersection of one primitive; updates the closest hit in `tr`.  Returns
// true when an occlusion query can stop.
template <bool STATS>
__device__ __forceinline__ bool prim_test(const float4 v0, const float4 e1, const float4 e2, int pi, Trav& tr,
                                          Counters& ct) {
  const float3 o = tr.o, d = tdir(tr);
  const int meta = __float_as_int(v0.w);
  float t, u = 0.0f, v = 0.0f;
  if (meta & 1) {  // triangle: Moller-Trumbore; u,v >= 0, u+v <= 1, 0 < t < tmax
    if (STATS) ct.tris++;
    const float det = mt_terms(o, d, f3(v0.x, v0.y, v0.z), f3(e1.x, e1.y, e1.z), f3(e2.x, e2.y, e2.z), u, v, t);
    if (det == 0.0f) return false;
    if (!(u >= 0.0f && v >= 0.0f && u + v <= 1.0f)) return false;
  } else {  // sphere, cancellation-free roots (Haines et al., Ray Tracing Gems ch.7)
    if (STATS) ct.spheres++;
    float3 fo = o - f3(v0.x, v0.y, v0.z);
    float bq = dot(fo, d);
    float3 lp = fo - d * bq;
    float disc = e1.y - dot(lp, lp);
    if (disc < 0.0f) return false;
    float q = -bq - copysignf(sqrtf(disc), bq);
    if (q == 0.0f) return false;
    float ta = (dot(fo, fo) - e1.y) / q, tb = q;
    float t1 = fminf(ta, tb), t2 = fmaxf(ta, tb);
    // nearest: nearer root unless behind the origin (sphere.cpp:47-77);
    // occlusion: the far root, as Sphere::intersect(r)'s aliased test (sphere.cpp:37-45)
    t = (t1 > 0.0f && !tr.any) ? t1 : t2;
  }
  if (t > 0.0f && t < tr.tmax) {
    tr.tmax = t;
    tr.prim = pi;
    tr.found = true;
    return tr.any;
  }
  return false;
}

// Traversal is split into two kinds of step so that a wave runs one kind at a
// time with most lanes active (if-if traversal with wave-level scheduling,
// after Aila & Laine 2009):
//  * node step (tr.node >= 0): fetch one 4-wide node (128 B), slab-test the
//    four child boxes, continue with the nearest child and push the others
//    farthest-first;
//  * leaf step (tr.node < 0, a leaf cursor): test up to two primitives of the
//    leaf with all six 16-B loads issued together, then pop.
// Children references (DNode.ref) are node indices or leaf cursors, so a
// leaf is entered, pushed and popped like a node.  Semantics: nearest hit
// (bvh.cpp:227-279, 343-362: the same closest hit, children visited near-first,
// boxes clipped to the current [0, tmax]) or, with tr.any, occlusion within
// (0, tmax) (bvh.cpp:282-341), leaving on the first hit.
// Per-lane traversal stack: the first PT_STACK entries in LDS (lane-
// contiguous, conflict-free), deeper ones in a global per-lane spill area that
// only BVHs with a worst-case depth beyond PT_STACK get (rarely touched).
// LDS pointers typed as such: a plain int* into __shared__ memory makes the
// compiler merge the LDS / spill paths into FLAT accesses, which occupy the
// vector-memory (TA/TD) path the node and primitive fetches need.
typedef __attribute__((address_space(3))) int lds_int;

struct Stack {
  lds_int* lds;   // s_stack + lane, stride PT_BLOCK
  int* spill;     // the spill area (wave-uniform base, may be null): column = global lane id, stride sstride
  uint32_t sstride;
  // Entry i >= PT_STACK of this lane.  The global lane id is re-derived at
  // each (rare) spill access from the workgroup id and the lane's mbcnt, in a
  // volatile asm the compiler cannot hoist: a per-lane 64-bit spill pointer
  // would hold two VGPRs in every wave for the whole kernel.
  __device__ __forceinline__ int* spill_at(int i) const {
    uint32_t l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return spill + ((size_t)(i - PT_STACK) * sstride + (size_t)blockIdx.x * PT_BLOCK + l);
  }
  __device__ __forceinline__ void put(int i, int v) const {
    if (i < PT_STACK) {
      lds[i * PT_BLOCK] = v;
    } else {
      *spill_at(i) = v;
    }
  }
  __device__ __forceinline__ int get(int i) const {
    int v;
    if (i < PT_STACK) {
      v = lds[i * PT_BLOCK];
    } else {
      v = *spill_at(i);
      // wait for the (rare) spill load here: otherwise the loop latch and
      // header wait vmcnt(0) for it on every iteration, and with it for the
      // group-sum stores the iteration issued (C3 +0.5%: r5/ab_sel_spill_compress.txt)
      asm volatile("" : "+v"(v));
    }
    return v;
  }
};

__device__ __forceinline__ bool trav_pop(const Stack& stk, Trav& tr) {
  if (tr.sp == 0) return true;
  --tr.sp;
  tr.node = stk.get(tr.sp);
  return false;
}

// Stack fast path: when no lane of the wave can touch the global spill area
// in this step (a wave-uniform ballot), pushes and pops are plain LDS
// accesses without per-lane branches: the divergent push / pop blocks, each
// with its own spill test, cost ~20 scalar instructions of exec-mask
// bookkeeping per traversal iteration, and a scalar instruction in the
// traversal loop costs more than a vector one (profiles/r5/probes_inst_cost.txt;
// C3 +1.5%: r5/ab_stack_fast_w8.txt).
// Pop for the lanes with `pop` set, every lane's stack top in LDS (sp <=
// PT_STACK); returns true for a lane whose stack was empty (its traversal is
// over).  The LDS read is issued for every lane (entry 0 for an empty stack).
__device__ __forceinline__ bool trav_pop_lds(const Stack& stk, Trav& tr, bool pop) {
  const int spm = max(tr.sp - 1, 0);
  const int top = stk.lds[spm * PT_BLOCK];
  const bool done = pop && tr.sp == 0;
  tr.node = pop ? top : tr.node;
  tr.sp = pop ? spm : tr.sp;
  return done;
}

__device__ __forceinline__ void cswap(float& da, int& ra, float& db, int& rb) {
  const bool sw = db < da;
  const float td = sw ? db : da;
  const int tr = sw ? rb : ra;  // references stay integers (leaf cursors exceed 2^24)
  db = sw ? da : db;
  rb = sw ? ra : rb;
  da = td;
  ra = tr;
}

// Child order of a node step: the full sort (5-exchange network, farthest
// pushed first).  Rays enter 1.02 children per node on average, so the order
// of the pushed ones hardly matters (CPU traversal census of the C3 ray mix,
// tools/wide_sim.cpp), and continuing with the nearest child while pushing
// the rest in slot order is a third of the network's VALU -- yet the network
// measured faster on the GPU (C3 +1.3%, C5 +1.8%: profiles/r5/ab_order_ballot.txt).
//
// Second half of a node step: entry distances d (kMiss = not entered) and
// references rf of the four children -> continue with the nearest, push the
// other hits.
__device__ __forceinline__ bool node_order(const Stack& stk, Trav& tr, const float* d, const int4 rf) {
  const float kMiss = 3.0e38f;
  int r0 = rf.x, r1 = rf.y, r2 = rf.z, r3 = rf.w;
  float d0 = d[0], d1 = d[1], d2 = d[2], d3 = d[3];
  // near-first order: 5-exchange sorting network on the entry distances
  cswap(d0, r0, d1, r1);
  cswap(d2, r2, d3, r3);
  cswap(d0, r0, d2, r2);
  cswap(d1, r1, d3, r3);
  cswap(d1, r1, d2, r2);
  if (__ballot(tr.sp > PT_STACK - 3) == 0ull) {  // (wave-uniform) three pushes and a pop stay in LDS
    // the hits are a sorted prefix: all three candidates are written, the top
    // advances past hits only; a lane that entered no child pushed nothing
    // and pops
    int sp = tr.sp;
    stk.lds[sp * PT_BLOCK] = r3;
    sp += d3 != kMiss;
    stk.lds[sp * PT_BLOCK] = r2;
    sp += d2 != kMiss;
    stk.lds[sp * PT_BLOCK] = r1;
    sp += d1 != kMiss;
    tr.sp = sp;
    tr.node = r0;
    const bool miss = d0 == kMiss;
    if (__ballot(miss) == 0ull) return false;
    return trav_pop_lds(stk, tr, miss);
  }
  if (d0 == kMiss) return trav_pop(stk, tr);
  // push the farther hits (farthest first), continue with the nearest.  The
  // hits are a sorted prefix, so with room for three entries every candidate
  // is written and the top only advances past hits (no branches).
  int sp = tr.sp;
  if (sp + 3 <= PT_STACK) {
    stk.lds[sp * PT_BLOCK] = r3;
    sp += d3 != kMiss;
    stk.lds[sp * PT_BLOCK] = r2;
    sp += d2 != kMiss;
    stk.lds[sp * PT_BLOCK] = r1;
    sp += d1 != kMiss;
  } else {
    if (d3 != kMiss) stk.put(sp++, r3);
    if (d2 != kMiss) stk.put(sp++, r2);
    if (d1 != kMiss) stk.put(sp++, r1);
  }
  tr.sp = sp;
  tr.node = r0;
  return false;
}

typedef __attribute__((address_space(3))) const char lds_cchar;
typedef float pt_v4f __attribute__((ext_vector_type(4)));
typedef int pt_v4i __attribute__((ext_vector_type(4)));
// 16-B LDS loads (ds_read_b128) into HIP vector types
__device__ __forceinline__ float4 lds_f4(lds_cchar* p) {
  const pt_v4f v = *(__attribute__((address_space(3))) const pt_v4f*)p;
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ int4 lds_i4(lds_cchar* p) {
  const pt_v4i v = *(__attribute__((address_space(3))) const pt_v4i*)p;
  return make_int4(v.x, v.y, v.z, v.w);
}

// Node step.  Near/far planes are chosen by the ray's direction signs through
// the load addresses: for inv.x >= 0 the near x plane is lo (offset 0), else
// hi (offset 16).  The slab test then needs no per-child min/max pairs:
// tn = max(near planes, 0), tf = min(far planes, tmax).  ROOT: the node is the
// workgroup's LDS copy of the root (`root`, ds_read_b128); otherwise the seven
// 16-B global loads are all issued before the first wait (register fence).
template <bool STATS, bool ROOT = false>
__device__ __forceinline__ bool node_step(const DNode* __restrict__ nodes, const Stack& stk, Trav& tr,
                                          Counters& ct, lds_cchar* root = nullptr) {
  const float kRobust = PT_ROBUST;
  const float3 o = tr.o, inv = tr.inv;
  const float kMiss = 3.0e38f;
  float d[4];
  const uint32_t sx = (__float_as_uint(inv.x) >> 27) & 16u, sy = (__float_as_uint(inv.y) >> 27) & 16u,
                 sz = (__float_as_uint(inv.z) >> 27) & 16u;
  float4 nx, fx, ny, fy, nz, fz;
  int4 rf;
  if constexpr (ROOT) {
    nx = lds_f4(root + sx);
    fx = lds_f4(root + (sx ^ 16u));
    ny = lds_f4(root + (32u + sy));
    fy = lds_f4(root + (32u + (sy ^ 16u)));
    nz = lds_f4(root + (64u + sz));
    fz = lds_f4(root + (64u + (sz ^ 16u)));
    rf = lds_i4(root + 96u);
  } else {
    const char* nb = (const char*)nodes;
    const uint32_t base = (uint32_t)tr.node << 7;
    nx = *(const float4*)(nb + (base + sx));
    fx = *(const float4*)(nb + (base + (sx ^ 16u)));
    ny = *(const float4*)(nb + (base + 32u + sy));
    fy = *(const float4*)(nb + (base + 32u + (sy ^ 16u)));
    nz = *(const float4*)(nb + (base + 64u + sz));
    fz = *(const float4*)(nb + (base + 64u + (sz ^ 16u)));
    rf = *(const int4*)(nb + (base + 96u));
    PT_FENCE4(fz);
    PT_FENCE4(rf);
  }
  if (STATS) ct.nodes++;
  const float3 oi = f3(o.x * inv.x, o.y * inv.y, o.z * inv.z);
  // (The 24 plane distances as packed v_pk_fma_f32 pairs -- half the FMA
  // issues, same roundings -- measured C3 -2.4%, C4 -1.9%, C5 -1.1%:
  // profiles/r4/ab_packed_node.txt)
  const float* NX = &nx.x; const float* FX = &fx.x; const float* NY = &ny.x;
  const float* FY = &fy.x; const float* NZ = &nz.x; const float* FZ = &fz.x;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float tn = fmaxf(fmaxf(fmaf(NX[k], inv.x, -oi.x), fmaf(NY[k], inv.y, -oi.y)),
                           fmaxf(fmaf(NZ[k], inv.z, -oi.z), 0.0f));
    const float tf = fminf(fminf(fmaf(FX[k], inv.x, -oi.x), fmaf(FY[k], inv.y, -oi.y)),
                           fminf(fmaf(FZ[k], inv.z, -oi.z), tr.tmax)) * kRobust;
    d[k] = tn <= tf ? tn : kMiss;
  }
  return node_order(stk, tr, d, rf);
}

// (Round 5 measured and removed two other node encodings: an 8-wide node with
// fp16 planes, C3 -8.2% / C4 -11.5% / C5 -9.8% -- more primitive tests and leaf
// steps than the 4-wide tree; and this 4-wide node compressed to fp16 planes
// from a node origin, 80 B, C3 -2.4%: profiles/r5/ab_stack_fast_w8.txt,
// ab_sel_spill_compress.txt; DESIGN.md "Why the wide node loses".)


// Binary node step over the reference topology (reference-count launch).
template <bool STATS>
__device__ __forceinline__ bool node_step2(const DNode2* __restrict__ nodes, const Stack& stk, Trav& tr,
                                           Counters& ct) {
  const float kRobust = PT_ROBUST;
  const float4 a = nodes[tr.node].a;
  const float4 b = nodes[tr.node].b;
  const float4 c = nodes[tr.node].c;
  const int4 e = nodes[tr.node].e;
  if (STATS) ct.nodes++;
  const float3 o = tr.o, inv = tr.inv;
  const float3 oi = f3(o.x * inv.x, o.y * inv.y, o.z * inv.z);
  float l0x = fmaf(a.x, inv.x, -oi.x), h0x = fmaf(a.y, inv.x, -oi.x);
  float l0y = fmaf(a.z, inv.y, -oi.y), h0y = fmaf(a.w, inv.y, -oi.y);
  float l0z = fmaf(c.x, inv.z, -oi.z), h0z = fmaf(c.y, inv.z, -oi.z);
  float l1x = fmaf(b.x, inv.x, -oi.x), h1x = fmaf(b.y, inv.x, -oi.x);
  float l1y = fmaf(b.z, inv.y, -oi.y), h1y = fmaf(b.w, inv.y, -oi.y);
  float l1z = fmaf(c.z, inv.z, -oi.z), h1z = fmaf(c.w, inv.z, -oi.z);
  float tn0 = fmaxf(fmaxf(fminf(l0x, h0x), fminf(l0y, h0y)), fmaxf(fminf(l0z, h0z), 0.0f));
  float tf0 = fminf(fminf(fmaxf(l0x, h0x), fmaxf(l0y, h0y)), fminf(fmaxf(l0z, h0z), tr.tmax)) * kRobust;
  float tn1 = fmaxf(fmaxf(fminf(l1x, h1x), fminf(l1y, h1y)), fmaxf(fminf(l1z, h1z), 0.0f));
  float tf1 = fminf(fminf(fmaxf(l1x, h1x), fmaxf(l1y, h1y)), fminf(fmaxf(l1z, h1z), tr.tmax)) * kRobust;
  bool in0 = tn0 <= tf0;
  bool in1 = tn1 <= tf1;
  if (in0 && in1) {
    bool first0 = tn0 <= tn1;
    stk.put(tr.sp, first0 ? e.y : e.x);
    ++tr.sp;
    tr.node = first0 ? e.x : e.y;
  } else if (in0) {
    tr.node = e.x;
  } else if (in1) {
    tr.node = e.y;
  } else {
    return trav_pop(stk, tr);
  }
  return false;
}

// Leaf cursor: ~((first << 3) | (count - 1)), count in [1, 8].
__device__ __forceinline__ int leaf_first(int cur) { return (~cur) >> 3; }
__device__ __forceinline__ int leaf_count(int cur) { return ((~cur) & 7) + 1; }

template <bool STATS, bool TRI = false>
__device__ __forceinline__ bool leaf_step(const DPrim* __restrict__ prims, const Stack& stk, Trav& tr,
                                          Counters& ct) {
  const int pa = leaf_first(tr.node);
  const int n = leaf_count(tr.node);
  const bool two = n >= 2;
  const int pb = two ? pa + 1 : pa;
  float4 a0 = prims[pa].v0, a1 = prims[pa].e1, a2 = prims[pa].e2;
  float4 b0 = prims[pb].v0, b1 = prims[pb].e1, b2 = prims[pb].e2;
  // One memory round trip per leaf step: without the fence the compiler sinks
  // the first primitive's e2 load into the triangle branch (a second
  // dependent L2 trip).  The fence makes the last-issued loads' values live
  // here, so every load is issued before the one wait.  (Skipping the second
  // triple for one-primitive steps measured -2%: the branch costs more.)
  PT_FENCE4(a2);
  PT_FENCE4(b2);
  if constexpr (TRI) {
    // Triangle-only scene: both Moller-Trumbore tests without branches (the
    // mixed build's per-primitive type test, det == 0 exit and sphere code
    // cost exec-mask bookkeeping in every leaf step).  Same predicate and
    // order as prim_test: the second triangle is tested against the tmax
    // the first left.  An occlusion ray that the first triangle already
    // stops may take the second one's (t, prim) as well -- only `found` is
    // read after an occlusion query.
    // (all six loads complete at one wait: without the fence the scheduler
    // waits for the first triple before it issues the second)
    PT_FENCE4(a0);
    PT_FENCE4(a1);
    PT_FENCE4(b0);
    PT_FENCE4(b1);
    const float3 o = tr.o, d = tdir(tr);
    float ua, va, ta, ub, vb, tb;
    const float da = mt_terms(o, d, f3(a0.x, a0.y, a0.z), f3(a1.x, a1.y, a1.z), f3(a2.x, a2.y, a2.z), ua, va, ta);
    const float db = mt_terms(o, d, f3(b0.x, b0.y, b0.z), f3(b1.x, b1.y, b1.z), f3(b2.x, b2.y, b2.z), ub, vb, tb);
    // (bitwise &: no short-circuit exec-mask blocks.)  Fewer compares, same
    // predicate: with det == 0 the reciprocal is inf and u, v are +-inf or
    // NaN, so u + v <= 1 and min(u, v) >= 0 cannot both hold -- the det test
    // is implied; and min(u, v) >= 0 differs from u >= 0 && v >= 0 only for a
    // NaN operand, where u + v <= 1 is false anyway.
    (void)da;
    (void)db;
    const bool ha = (fminf(ua, va) >= 0.0f) & (ua + va <= 1.0f) & (ta > 0.0f) & (ta < tr.tmax);
    const float tm = ha ? ta : tr.tmax;
    const bool hb = two & (fminf(ub, vb) >= 0.0f) & (ub + vb <= 1.0f) & (tb > 0.0f) & (tb < tm);
    tr.tmax = hb ? tb : tm;
    tr.prim = hb ? pb : ha ? pa : tr.prim;
    tr.found = tr.found || ha || hb;
    if (STATS) ct.tris += two ? 2u : 1u;
    if (__ballot(tr.sp > PT_STACK) == 0ull) {  // (wave-uniform) every pop reads LDS
      const bool stop = tr.any & (ha | hb);   // occlusion found: the ray is done
      const bool more = n > 2;                // the leaf's next two primitives
      tr.node = more ? ~(((pa + 2) << 3) | (n - 3)) : tr.node;
      const bool pop = !stop & !more;
      if (__ballot(pop) == 0ull) return stop;
      return stop | trav_pop_lds(stk, tr, pop);
    }
    if (tr.any && (ha || hb)) return true;
  } else {
    if (prim_test<STATS>(a0, a1, a2, pa, tr, ct)) return true;
    if (two && prim_test<STATS>(b0, b1, b2, pb, tr, ct)) return true;
  }
  if (n > 2) {
    tr.node = ~(((pa + 2) << 3) | (n - 3));
    return false;
  }
  return trav_pop(stk, tr);
}

template <bool STATS>
__device__ __forceinline__ bool trav_step(const DNode* __restrict__ nodes, const DPrim* __restrict__ prims,
                                          const Stack& stk, Trav& tr, Counters& ct) {
  return tr.node < 0 ? leaf_step<STATS>(prims, stk, tr, ct) : node_step<STATS>(nodes, stk, tr, ct);
}

template <bool STATS>
__device__ __forceinline__ bool traverse(const DNode* __restrict__ nodes, const DPrim* __restrict__ prims,
                                         const Stack& stk, float3 o, float3 d,
                                         float tmax, bool any, Hit& hit, Counters& ct) {
  Trav tr;
  trav_init(tr, o, d, tmax, any);
  while (!trav_step<STATS>(nodes, prims, stk, tr, ct)) {
  }
  hit.t = tr.tmax;
  hit.prim = tr.prim;
  return tr.found;
}

// Robust slab test of the ray in `tr` against one box (lo, hi), clipped to [0, tmax].
template <class T>
__device__ __forceinline__ bool box_hit(const Trav& tr, const T* lo, const T* hi) {
  const float3 oi = f3(tr.o.x * tr.inv.x, tr.o.y * tr.inv.y, tr.o.z * tr.inv.z);
  float lx = fmaf(lo[0], tr.inv.x, -oi.x), hx = fmaf(hi[0], tr.inv.x, -oi.x);
  float ly = fmaf(lo[1], tr.inv.y, -oi.y), hy = fmaf(hi[1], tr.inv.y, -oi.y);
  float lz = fmaf(lo[2], tr.inv.z, -oi.z), hz = fmaf(hi[2], tr.inv.z, -oi.z);
  float tn = fmaxf(fmaxf(fminf(lx, hx), fminf(ly, hy)), fmaxf(fminf(lz, hz), 0.0f));
  float tf = fminf(fminf(fmaxf(lx, hx), fmaxf(ly, hy)), fminf(fmaxf(lz, hz), tr.tmax)) * PT_ROBUST;
  return tn <= tf;
}

// ---- EnvironmentLight (src/static_scene/environment_light.cpp), fp32.
// sample_dir (130-199): lat-long bilinear lookup at texel coordinates (tu,
// tv), wrapping in both directions exactly as the reference does.
template <class KP>
__device__ __forceinline__ float3 env_uv(const KP& P, float tu, float tv) {
  const int w = P.env_w, h = P.env_h;
  const int su = (int)tu, sv = (int)tv;
  float a, b;
  int px1, px2, py1, py2;
  if (tu < 0.0f) {
    a = tu + 1.0f; px1 = w - 1; px2 = 0;
  } else if (tu >= (float)(w - 1)) {
    a = tu - (float)w + 1.0f; px1 = w - 1; px2 = 0;
  } else {
    a = tu - (float)su; px1 = su; px2 = su + 1;
  }
  if (tv < 0.0f) {
    b = tv + 1.0f; py1 = h - 1; py2 = 0;
  } else if (tv >= (float)(h - 1)) {
    b = tv - (float)h + 1.0f; py1 = h - 1; py2 = 0;
  } else {
    b = tv - (float)sv; py1 = sv; py2 = sv + 1;
  }
  const float4 z11 = P.env_tex[px1 + w * py1], z21 = P.env_tex[px2 + w * py1];
  const float4 z12 = P.env_tex[px1 + w * py2], z22 = P.env_tex[px2 + w * py2];
  const float3 zy1 = f3(z11.x, z11.y, z11.z) * (1.0f - a) + f3(z21.x, z21.y, z21.z) * a;
  const float3 zy2 = f3(z12.x, z12.y, z12.z) * (1.0f - a) + f3(z22.x, z22.y, z22.z) * a;
  return zy1 * (1.0f - b) + zy2 * b;
}

// sample_dir of a direction: (theta, phi) from the direction, then the lookup
template <class KP>
__device__ __forceinline__ float3 env_dir(const KP& P, float3 d) {
  const float kPi = 3.14159265358979323f;
  const int w = P.env_w, h = P.env_h;
  const float theta = acosf(fminf(fmaxf(d.y, -1.0f), 1.0f));
  const float sin_theta = fsqrt(fmaxf(0.0f, 1.0f - d.y * d.y));
  float phi = sin_theta == 0.0f ? kPi : acosf(fminf(fmaxf(d.z / sin_theta, -1.0f), 1.0f));
  if (d.x > 0.0f) phi = 2.0f * kPi - phi;
  const float tu = phi * (0.15915494309189535f * (float)w) - 0.5f;
  const float tv = theta * (0.31830988618379067f * (float)h) - 0.5f;
  return env_uv(P, tu, tv);
}

// importanceSampling (69-115): inverse CDF over rows (pTheta), then within the
// row (pPhiGivenTheta), linear inside the texel; pdf per solid angle.
// The sampled direction's radiance (sample_L returns sample_dir(wi)) is
// looked up at the texel coordinates the sample was drawn at, (x - 0.5,
// y - 0.5) -- what sample_dir's acos round trip of wi yields up to float
// rounding (~1e-5 texel), without its two acosf and a division on the
// NEE's dependent chain: returned in (tu, tv) for env_uv (C5 +1.5%:
// profiles/r4/ab_env_uv_groups.txt).
template <class KP>
__device__ __forceinline__ void env_sample(const KP& P, float r1, float r2, float3& wi, float& pdf, float& tu,
                                           float& tv) {
  const float kPi = 3.14159265358979323f;
  const int w = P.env_w, h = P.env_h;
  const float u1 = r1;
  r1 *= P.env_ptheta[h - 1];
  float prev, cur;
  const int t = record_lower_bound(P.env_ptheta, r1, u1, P.env_rtheta, PT_ENV_GUIDE, prev, cur);
  const float y = (float)t + (r1 - prev) / (cur - prev);
  tv = fminf(y, (float)h) - 0.5f;
  const float theta = fminf(y / (float)h, 1.0f) * kPi;
  const float* row = P.env_pphi + (size_t)t * w;
  const float u2 = r2;
  r2 *= row[w - 1];
  const int q = record_lower_bound(row, r2, u2, P.env_rphi + (size_t)t * PT_ENV_GUIDE, PT_ENV_GUIDE, prev, cur);
  const float x = (float)q + (r2 - prev) / (cur - prev);
  tu = fminf(x, (float)w) - 0.5f;
  const float phi = fminf(x / (float)w, 1.0f) * (2.0f * kPi);
  float st, ct, sp, cp;
  __sincosf(theta, &st, &ct);
  __sincosf(phi, &sp, &cp);
  pdf = P.env_pdf[(size_t)t * w + q] / (st * ((2.0f * kPi / (float)w) * (kPi / (float)h)));
  wi = f3(-st * sp, ct, st * cp);
}

// Lane modes of the persistent kernel.
enum : int { M_TRAV = 0, M_SHADE = 1, M_FETCH = 2, M_CAMERA = 3, M_DONE = 4 };
// What follows a lane's shadow ray (the `shadow` state; 0 = not a shadow ray).
enum : int { SH_HELPER = -1, SH_RESUME = 1, SH_FOLLOW = 2, SH_STORE = 3, SH_STORE_FOLLOW = 4 };
// Wave priorities of the two phases (s_setprio; shading raised: round 3,
// profiles/r3/ab_build_options.txt)
#ifndef PT_PRIO_SHADE
#define PT_PRIO_SHADE 2
#endif
#ifndef PT_PRIO_TRAV
#define PT_PRIO_TRAV 0
#endif

// Wave-clock sections of the STATS build: every shader clock of a wave's
// lifetime falls in exactly one (pt_stats.shade_clocks + trav_clocks = the
// waves' summed lifetimes; section_clocks = S_HIT .. S_FETCH).
enum : int { S_HIT = 0, S_NEE = 1, S_BSDF = 2, S_FETCH = 3, S_CAMERA = 4, S_TRAV = 5, S_OTHER = 6, S_N = 7 };

// DBG: diagnostic build that printf-traces the pixel P.dbg_pix (PT_DEBUG_PIXEL=x,y)
// Occupancy target: 5 waves per SIMD = at most 96 VGPRs (512 / 5, granule 8)
// and 8 KB of LDS per wave (160 KB / 20 waves per CU; the 24-entry stack is
// 6 KB).  The traversal is latency-bound, so waves per SIMD pay directly:
// C3 16.0 / 20.5 / 23.6 / 24.9 Gsamples/s at 2 / 3 / 4 / 5 waves per SIMD.
#ifndef PT_MIN_WAVES_PER_SIMD
#define PT_MIN_WAVES_PER_SIMD 5
#endif
// BIN: the reference-count variant, traversing the binary tree (P.nodes2).
// ENV: the scene has an environment light (kept out of the common build: its
// lookups and sampling cost registers).
// GTAB: material/light tables larger than the LDS copies (read from global
// memory; the common build reads them from LDS through address-space-typed
// pointers, never through FLAT accesses).
// TRI: every primitive is a triangle (branch-free leaf steps, no sphere test).
// MF: a frame batch (KParams.n_frames frames of one tile set in one launch,
// plain common build only): the queue runs over every frame's work slots, so
// a small frame's drain is filled by the next frame's slots.
template <bool STATS, bool DBG, bool BIN, bool ENV, bool GTAB, bool TRI = false, bool MF = false>
__global__ __launch_bounds__(PT_BLOCK, PT_MIN_WAVES_PER_SIMD) void render_kernel(KParams P) {
  // the wave's PT_STACK x 64 LDS stack (lane-contiguous rows)
  __shared__ int s_stack[PT_STACK * PT_BLOCK];
  const int lane = threadIdx.x;
  const uint32_t wave_id = blockIdx.x;  // the persistent wave (one per workgroup)
  const uint32_t n_waves = gridDim.x;
  const Stack stk{(lds_int*)(s_stack + lane), P.stack_spill, n_waves * PT_BLOCK};
  // The BVH4 root, which every ray visits first: one LDS copy per wave, so
  // the root step of a fresh ray costs no vector-memory traffic (C3 +2%).
  __shared__ int4 s_root[sizeof(DNode) / 16];
  if (!BIN) {
    if (lane < 8) s_root[lane] = ((const int4*)P.nodes)[lane];
  }

  // Material and light tables are read by every shading step: keep small
  // ones in LDS (the usual case); larger ones stay in global memory.
  __shared__ DBsdf s_bsdf[GTAB ? 1 : PT_LDS_BSDFS];
  __shared__ DLight s_light[GTAB ? 1 : PT_LDS_LIGHTS];
  typedef __attribute__((address_space(3))) const float lds_f;
  if (!GTAB) {
    const int nb = P.n_bsdfs * (int)(sizeof(DBsdf) / 4);
    for (int k = lane; k < nb; k += PT_BLOCK) ((float*)s_bsdf)[k] = ((const float*)P.bsdfs)[k];
    const int nl = P.n_lights * (int)(sizeof(DLight) / 4);
    for (int k = lane; k < nl; k += PT_BLOCK) ((float*)s_light)[k] = ((const float*)P.lights)[k];
  }
  // Table fields are read where they are used (address-space-typed ds_read
  // loads in the LDS build), never copied whole into registers: every value
  // live in the shading code costs a VGPR in all waves.
  auto bsdf_f = [&](int i, int k) -> float {
    if constexpr (GTAB) return ((const float*)P.bsdfs)[i * (int)(sizeof(DBsdf) / 4) + k];
    else return ((lds_f*)s_bsdf)[i * (int)(sizeof(DBsdf) / 4) + k];
  };
  auto light_f = [&](int i, int k) -> float {
    if constexpr (GTAB) return ((const float*)P.lights)[i * (int)(sizeof(DLight) / 4) + k];
    else return ((lds_f*)s_light)[i * (int)(sizeof(DLight) / 4) + k];
  };
#define PT_BSDF3(i, field) f3(bsdf_f(i, offsetof(DBsdf, field) / 4), bsdf_f(i, offsetof(DBsdf, field) / 4 + 1), bsdf_f(i, offsetof(DBsdf, field) / 4 + 2))
#define PT_LIGHT3(i, field) f3(light_f(i, offsetof(DLight, field) / 4), light_f(i, offsetof(DLight, field) / 4 + 1), light_f(i, offsetof(DLight, field) / 4 + 2))
  // STATS: the wave's clock sections and its last stamp, in LDS.  A stamp is
  // written by the first ACTIVE lane, so stamps inside divergent shading code
  // account the wave's time whichever lanes took the branch.
  __shared__ unsigned long long s_clk[STATS ? S_N + 1 : 1];
  if (STATS && lane <= S_N) s_clk[lane] = lane == S_N ? clock64() : 0ull;
  // STATS: work-slot latency histogram (log2 of microseconds, 32 buckets)
  __shared__ uint32_t s_hist[STATS ? 32 : 1];
  if (STATS && lane < 32) s_hist[lane] = 0u;
  __syncthreads();
  // From here on the launch parameters are read through a pointer to the
  // kernel-argument segment that an empty asm "changes" at the start of every
  // round: their scalar loads stay inside the round (scalar-cache hits)
  // instead of being hoisted to the kernel's start and held in SGPRs for the
  // whole kernel -- spilled SGPRs occupy VGPR lanes, and the constants the
  // SGPR allocator then keeps in VGPRs cost the ENV build its spills (C5
  // +6.8%, C3 +0.9%: profiles/r3/ab_kernarg_round.txt, r4/ab_layout.txt).
  typedef __attribute__((address_space(4))) const KParams karg_t;
  karg_t* Q = (karg_t*)__builtin_amdgcn_kernarg_segment_ptr();
#define P (*Q)
#define PT_STAMP(k)                                                  \
  if constexpr (STATS) {                                             \
    const unsigned long long t_ = clock64();                         \
    if (lane == __builtin_amdgcn_readfirstlane(lane)) {              \
      s_clk[k] += t_ - s_clk[S_N];                                   \
      s_clk[S_N] = t_;                                               \
    }                                                                \
  }

  // ---- per-lane state
  int mode = M_FETCH;
  // the ray in flight: 0 extension (camera / bounce) ray, else a shadow ray
  // followed by -- SH_RESUME: the shading round (NEE resumes at the cursor);
  // SH_FOLLOW: the next extension ray, already sampled (origin in hp,
  // direction in ns), started inside the traversal loop; SH_STORE: the
  // group already ended and the lane was refilled -- acc keeps the group's
  // total without the light sample, pend the total with it, and ONE store at
  // oslot writes the right one when the shadow ray ends; then the lane
  // retires (the queue is drained) or, with SH_STORE_FOLLOW, goes on with the
  // next group's camera ray parked in (hp, ns).  While a store is pending the
  // new group's sum (the environment its missed camera rays saw) gathers in
  // ng, which is dead between a path's last vertex and the next hit record.
  int shadow = 0;
  uint32_t oslot = 0;
  // (drain helpers) the lane tracing this lane's last shadow ray, -1 for none
  int hl = -1;
  // the work slot (pixel, sample group) this lane renders: its index (where
  // the group's sum goes), its pixel as packed coordinates (x | y << 16;
  // W, H <= 65535) and its current sample
  uint32_t myslot = 0;
  int pix = 0, sample = 0;
  // the sample's stream and the counter word of its next draw (ptrng::draw_at)
  uint32_t rbase = 0, rdim = ptrng::kDrawInit;
#define PT_DRAW() ptrng::draw_at(rbase, (rdim += ptrng::kDrawStep) - ptrng::kDrawStep)
  float3 acc = f3(0, 0, 0);  // the slot's radiance sum: each path contribution is added as it is found
  float3 T = f3(1, 1, 1);    // path throughput
  // path depth (bits 0-7) and the NEE cursor: light sample (8-15), light
  // index (16-31), packed in one register -- they persist across traversal,
  // where every register counts (max_depth <= 254, ns_area_light <= 255,
  // lights < 65536: pt_set_params / pt_upload_scene check)
  uint32_t cur = 0;
  bool includeLe = true;
  // shading record of the current path vertex
  float3 hp = f3(0, 0, 0), ns = f3(0, 0, 1), ng = f3(0, 0, 1);
  int bsdf = 0;
  float3 pend = f3(0, 0, 0);  // NEE contribution awaiting its shadow ray
  Trav tr;
  trav_init(tr, f3(0, 0, 0), f3(0, 0, 1), 0.0f, false);
  Counters ct = {0, 0, 0};
  uint32_t n_cam = 0, n_bounce = 0, n_shadow = 0, n_hits = 0;
  uint32_t n_titer = 0, n_rounds = 0;  // wave-level traversal steps / shading rounds (lane 0)
  uint32_t n_leafit = 0;               // of the traversal steps: leaf steps
  // traversal lane-iterations: at the other step kind, finished and waiting
  // for the shading round, retired, stepping a leaf
  uint32_t l_other = 0, l_ready = 0, l_dead = 0, l_leaf = 0;
  uint32_t l_deep = 0;  // traversal lane-steps taken with stack entries in the global spill area
  // node-step census (STATS, wave-uniform): main-loop wave node steps, of them
  // with every stepping lane at ONE node, lanes at the first lane's node,
  // stepping lanes, steps / lanes inside the top two / three BVH4 levels
  // below the root (breadth-first node order: indices < 21 / < 85)
  uint32_t c_wsteps = 0, c_uniform = 0, c_cover = 0, c_lanes = 0, c_top2w = 0, c_top2l = 0, c_top3w = 0,
           c_top3l = 0;
  uint32_t n_atomics = 0;              // work-queue atomics (lane 0)
  uint32_t n_titer_drain = 0, n_rounds_drain = 0;  // of them: after this wave found the queue empty
  uint32_t chunk_next = 0, chunk_end = 0;  // the wave's private range of work slots
  uint32_t seen = 0;                       // queue head after this wave's last claim
  bool first_claim = true;                 // the first chunk is the wave's own (no atomic)
  // the queue head this wave claims from: its XCD's (HW_REG_XCC_ID), until that one runs dry
  uint32_t qh = (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | 20) % PT_QUEUE_HEADS;
  const unsigned long long w_start = STATS ? wall_clock64() : 0ull;
  // Residency census of the plain build (PT_CENSUS set, diagnostics): when
  // each wave started and ended, and where it ran -- which waves of the grid
  // were resident from the start; with a -DPT_CENSUS=1 build also its drain.
  unsigned long long* const census = (!STATS && P.census) ? P.stats + PT_STATS_SLOTS + PT_WAVE_TRACE * (size_t)wave_id : nullptr;
  if (census && lane == 0) {
    census[0] = wall_clock64();
    census[3] = ((unsigned long long)__builtin_amdgcn_s_getreg((3 << 11) | 20) << 32) |
                (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
  }
  unsigned long long w_empty = 0ull;  // when this wave first found the queue empty
#if PT_CENSUS
  int census_alive = -1, census_rounds = 0;  // (census: lanes alive at the drain's first round, rounds since)
  unsigned long long census_claim = 0ull, census_claim_max = 0ull;  // (census: wall ticks waiting on queue claims)
  uint32_t census_claims = 0;
#endif
  unsigned long long slot_t0 = 0ull, slot_lat_sum = 0ull, slot_lat_max = 0ull;  // work-slot latency (wall ticks)
  // per ray: traversal iterations it stepped in / sat out, traversal phases it spanned
  uint32_t r_steps = 0, r_idle = 0, r_rounds = 0, ray_steps_max = 0, ray_idle_max = 0, ray_rounds_max = 0;
#define PT_SLOT_DONE()                                                          \
  if (STATS) {                                                                  \
    const unsigned long long d_ = wall_clock64() - slot_t0;                    \
    slot_lat_sum += d_;                                                         \
    slot_lat_max = d_ > slot_lat_max ? d_ : slot_lat_max;                       \
    const uint32_t us_ = (uint32_t)min(d_ / 100ull, 0xffffffffull);            \
    const uint32_t b_ = us_ == 0u ? 0u : min(31u, 32u - (uint32_t)__clz(us_)); \
    atomicAdd(&s_hist[b_], 1u);                                                 \
  }

  // the lane's group ends before sample s (a shift when group_spp is a power
  // of two, the usual case; wave-uniform branch; the last group may be short)
  auto group_ends = [&](int s) -> bool {
    return s >= P.spp || (P.group_shift >= 0 ? (s & (P.group_spp - 1)) == 0 : s % P.group_spp == 0);
  };
  // the pixel index from the packed coordinates: one multiply-add, no
  // division per camera ray
  auto pix_index = [&](int p) -> int { return (p & 0xffff) + (int)((uint32_t)p >> 16) * P.W; };
  const uint32_t total_slots = (uint32_t)P.n_blocks * 64u * (uint32_t)P.n_groups * (MF ? (uint32_t)P.n_frames : 1u);
  const int batch = P.shade_batch;
  // Camera::generate_ray (camera.cpp:113-129) for the lane's pixel and
  // current sample, at the jittered position of raytrace_pixel
  // (pathtracer.cpp:571-575); starts the sample's random stream.  Returns
  // whether the ray enters the scene's root box (a ray that misses it sees
  // nothing but the environment: pathtracer.cpp:421-426).
  auto camera_ray = [&](Trav& t, float3& d) -> bool {
    const int px = pix & 0xffff, py = (int)((uint32_t)pix >> 16);
    uint32_t seed = P.seed;
    if constexpr (MF) {  // the lane's frame of the batch keys its samples
      const uint32_t f = pt_fastdiv(myslot, P.frm_m, P.frm_sh);
      seed = P.seeds[0];
#pragma unroll
      for (int i = 1; i < PT_MAX_FRAMES; ++i) seed = f == (uint32_t)i ? P.seeds[i] : seed;
    }
    rbase = ptrng::stream_base(seed, (uint32_t)(px + py * P.W), (uint32_t)sample + P.sample_base);
    rdim = ptrng::kDrawInit;
    float ry = PT_DRAW();  // UniformGridSampler2D draws y first
    float rx = PT_DRAW();
    float fx = ((float)px + rx) * P.inv_w;
    float fy = ((float)py + ry) * P.inv_h;
    float3 sp = f3((0.5f - fx) * P.cam_ax, (0.5f - fy) * P.cam_ay, 1.0f);
    float3 wsp = ld3(P.c2w_col0) * sp.x + ld3(P.c2w_col1) * sp.y + ld3(P.c2w_col2) * sp.z;
    d = normalize(f3(0, 0, 0) - wsp);
    trav_init(t, wsp + ld3(P.cam_pos), d, 3.0e38f, false);
    if (STATS) n_cam++;
    if (DBG && pix_index(pix) == P.dbg_pix) printf("pixel (%d,%d) sample %d o=(%.9g %.9g %.9g) d=(%.9g %.9g %.9g)\n", px, py, sample, t.o.x, t.o.y, t.o.z, d.x, d.y, d.z);
    return box_hit(t, P.root_lo, P.root_hi);
  };

  // A shadow ray ended (`done`) with what follows it already settled: add the
  // light sample (or store the group's total with it) and go on with the
  // next extension ray -- or retire -- without a shading round.
  auto follow_on = [&](bool done) {
    {  // (the divergent branch alone skips itself when no lane takes it)
      if (done && shadow >= SH_FOLLOW) {
        if (shadow == SH_FOLLOW) {
          if (!tr.found) acc = acc + pend;
        } else {  // the finished group's one store: its total with the light sample if the shadow ray is clear
          store_sum(P.partial + 3 * (size_t)oslot, tr.found ? acc : pend);
          acc = ng;  // the new group's sum so far (environment seen by its camera rays that missed)
        }
        if (shadow == SH_STORE) {
          mode = M_DONE;
        } else {
          Trav nt;
          trav_init(nt, hp, ns, 3.0e38f, false);
          tr.o = nt.o;
          tr.d = nt.d;
          tr.inv = nt.inv;
          tr.any = false;
          mode = M_TRAV;
        }
        shadow = 0;
      }
    }
    // the follow-up ray's traversal state by selects, outside the branch: the
    // loop-carried node / stack / tmax / primitive keep one register each
    // (with the branch the compiler copied them to and fro every iteration;
    // C3 +0.7%: profiles/r5/ab_helpers_followsel.txt)
    const bool fo = done && mode == M_TRAV;
    tr.node = fo ? 0 : tr.node;
    tr.sp = fo ? 0 : tr.sp;
    tr.tmax = fo ? 3.0e38f : tr.tmax;
    tr.prim = fo ? -1 : tr.prim;
    tr.found = fo ? false : tr.found;
  };

  for (;;) {
    asm volatile("" : "+s"(Q));
    // the shading round issues at raised wave priority, traversal at the
    // base one (C4 +0.6%, C5 +0.4%, C3 within noise: profiles/r3/ab_build_options.txt)
    __builtin_amdgcn_s_setprio(PT_PRIO_SHADE);
    // Drain helpers (the pairing is at the end of the refill): a helper's
    // shadow ray ended -- its owner adds the light sample if the ray was
    // clear, before anything else of its path (the order of trace_ray's
    // additions is kept), and the helper retires again.  An owner whose path
    // ray ended first waits in M_SHADE until then.
    if constexpr (!DBG && !BIN) {
      const bool hdone = shadow == SH_HELPER && mode == M_SHADE;
      const unsigned long long hd = __ballot(hdone);
      if (hd != 0ull) {  // (wave-uniform)
        const unsigned long long hc = __ballot(hdone && !tr.found);
        if (hl >= 0 && ((hd >> hl) & 1ull)) {
          if ((hc >> hl) & 1ull) acc = acc + pend;
          hl = -1;
        }
        if (hdone) {
          mode = M_DONE;
          shadow = 0;
        }
      }
    }
    // ================= shading phase: lanes whose ray finished =================
    if (mode == M_SHADE && hl < 0) {
      const bool found = tr.found;
      bool finish = false;  // the sample is complete
      bool group_end = false;  // the group's last sample ended: store its sum
      bool after = false;      // the sample's last shadow ray is emitted: the bounce / camera ray follows it
      int stage;            // 0: NEE (+ bounce), 2: none
      if (shadow) {  // (SH_RESUME: the follow-ups end inside the traversal loop)
        if (!found) acc = acc + pend;  // unoccluded (the light sample was already counted)
        if (DBG && pix_index(pix) == P.dbg_pix) printf("    shadow %s (pend %.6g) prim %d t %.9g\n", found ? "occluded" : "clear", pend.x, tr.prim, tr.tmax);
        stage = 0;
        shadow = 0;
      } else if (!found) {
        // miss: the environment map if there is one and includeLe (pathtracer.cpp:411-427)
        if (ENV && includeLe) acc = acc + mul(T, env_dir(P, tdir(tr)));
        finish = true;
        stage = 2;
      } else {
        if (STATS) n_hits++;
        // ---- hit record (Intersection, trace_ray lines 435-456).  Hit points
        // are rebuilt from the primitive (barycentrics / sphere reprojection),
        // not o + t*d, so their error is relative to the primitive and the
        // 256-ulp origin offset always clears the surface.  The whole record
        // and the vertex normals are fetched in one memory round trip
        // (unfenced, the e1/e2 and normal loads wait behind the meta branch).
        DPrim pr = P.prims[tr.prim];
        float nn[9];
        for (int k = 0; k < 9; ++k) nn[k] = P.norms[9 * (size_t)tr.prim + k];
        PT_FENCE4(pr.e2);
        asm volatile("" : "+v"(nn[8]));
        const int meta = __float_as_int(pr.v0.w);  // (bsdf << 1) | is_triangle
        bsdf = meta >> 1;
        if (meta & 1) {
          float3 V0 = f3(pr.v0.x, pr.v0.y, pr.v0.z), E1 = f3(pr.e1.x, pr.e1.y, pr.e1.z), E2 = f3(pr.e2.x, pr.e2.y, pr.e2.z);
          float hu, hv, ht;
          mt_terms(tr.o, tdir(tr), V0, E1, E2, hu, hv, ht);  // the barycentrics of the traversal test
          float w0 = 1.0f - hu - hv;
          hp = V0 + E1 * hu + E2 * hv;
          ns = ld3(nn) * w0 + ld3(nn + 3) * hu + ld3(nn + 6) * hv;
          ng = cross(E1, E2);
        } else {
          float3 C = f3(pr.v0.x, pr.v0.y, pr.v0.z);
          ns = normalize(tr.o + tdir(tr) * tr.tmax - C);
          hp = C + ns * pr.e1.x;
          ng = ns;
        }
        // Triangle::intersect flips the shading normal to face the ray
        // (triangle.cpp:95-99); Sphere::intersect keeps it outward
        // (sphere.cpp:66-70), which is what tells GlassBSDF a ray is leaving.
        if ((meta & 1) && dot(tdir(tr), ns) > 0.0f) ns = f3(0, 0, 0) - ns;
        ng = normalize(ng);
        if (includeLe) acc = acc + mul(T, PT_BSDF3(bsdf, e));
        if (DBG && pix_index(pix) == P.dbg_pix) printf("  depth %d hit prim %d bsdf %d t=%.9g n=(%.6g %.6g %.6g) T=(%.5g)\n", (int)(cur & 0xffu), tr.prim, bsdf, tr.tmax, ns.x, ns.y, ns.z, T.x);
        cur &= 0xffu;  // NEE starts at light 0, sample 0
        stage = 0;
      }
      PT_STAMP(S_HIT);
      if (stage < 2) {
        const int btype = __float_as_int(bsdf_f(bsdf, 0));
        const Frame fr = make_frame(ns);
        bool emitted = false;
        // ---- next-event estimation over all lights (pathtracer.cpp:469-523),
        // one light sample per shading round: the lane leaves with the sample's
        // shadow ray and resumes at the cursor when it returns
        int li = (int)(cur >> 16), ls = (int)((cur >> 8) & 0xffu);
        while (li < P.n_lights) {
          const int ltype = __float_as_int(light_f(li, 0));
          const bool delta = ltype == 0 || ltype == 2;
          const int nls = delta ? 1 : P.ns_area;
          if (ls >= nls) {
            ++li;
            ls = 0;
            continue;
          }
          float3 wi;
          float dist, pdf;
          float etu = 0.0f, etv = 0.0f;  // (environment light: the sample's texel coordinates)
          bool lit = true;
          if (ENV && ltype == 4) {  // EnvironmentLight::sample_L (environment_light.cpp:117-128)
            float r1 = PT_DRAW();
            float r2 = PT_DRAW();
            env_sample(P, r1, r2, wi, pdf, etu, etv);
            dist = 3.0e38f;
          } else if (ltype == 3) {  // AreaLight::sample_L (light.cpp:80-92); grid sampler draws y first
            float u0 = PT_DRAW();
            float u1 = PT_DRAW();
            float sx = u1 - 0.5f, sy = u0 - 0.5f;
            float3 dv = PT_LIGHT3(li, pos) + PT_LIGHT3(li, dimx) * sx + PT_LIGHT3(li, dimy) * sy - hp;
            float cosL = dot(dv, PT_LIGHT3(li, dir));
            float sq = dot(dv, dv);
            dist = fsqrt(sq);
            wi = dv * rcp(dist);
            pdf = sq * rcp(light_f(li, offsetof(DLight, area) / 4) * fabsf(cosL));  // unnormalised d.dir, as the reference
            lit = cosL < 0.0f;
          } else if (ltype == 1) {  // InfiniteHemisphereLight (light.cpp:34-42)
            float r1 = PT_DRAW();
            float r2 = PT_DRAW();
            float st = fsqrt(fmaxf(0.0f, 1.0f - r1 * r1));
            wi = f3(st * cos_rev(r2), r1, -st * sin_rev(r2));  // phi = 2 pi r2
            dist = 3.0e38f;
            pdf = 0.15915494309189535f;
          } else if (ltype == 2) {  // PointLight (light.cpp:49-57)
            float3 dv = PT_LIGHT3(li, pos) - hp;
            dist = fsqrt(dot(dv, dv));
            wi = dv * rcp(dist);
            pdf = 1.0f;
          } else {  // DirectionalLight (light.cpp:17-23)
            wi = PT_LIGHT3(li, dir);
            dist = 3.0e38f;
            pdf = 1.0f;
          }
          // (float)(1.0 / num_light_samples) (pathtracer.cpp:481), from the host
          const float scale = delta ? 1.0f : P.nls_scale;
          ++ls;
          // f() is zero for every BSDF but Diffuse (bsdf.cpp:34-202): nothing to add.
          if (btype != 0 || !lit) continue;
          float cos_t = fmaxf(0.0f, fr.to_local(wi).z);
          if (!(cos_t > 0.0f)) continue;
          float3 f = PT_BSDF3(bsdf, a) * 0.31830988618379067f;
          const float3 Le = (ENV && ltype == 4) ? env_uv(P, etu, etv)
                                                : PT_LIGHT3(li, rad);
          pend = mul(mul(T, Le * (cos_t * rcp(pdf))), f) * scale;
          // shadow ray (pathtracer.cpp:497-504): delta lights offset EPS_N along n
          float3 so = delta ? hp + ns * 5e-3f : offset_ray(hp, dot(wi, ng) >= 0.0f ? ng : f3(0, 0, 0) - ng);
          trav_init(tr, so, wi, dist * 0.999f, true);
          if (DBG && pix_index(pix) == P.dbg_pix) printf("    shadow o=(%.9g %.9g %.9g) d=(%.9g %.9g %.9g) maxt=%.9g cos %.4g pdf %.4g\n", so.x, so.y, so.z, wi.x, wi.y, wi.z, tr.tmax, cos_t, pdf);
          emitted = true;
          if (STATS) n_shadow++;
          break;
        }
        // the shadow ray just emitted is the vertex's last light sample
        const bool emit_last = emitted && li + 1 >= P.n_lights &&
                               ls >= ((__float_as_int(light_f(li, 0)) | 2) == 2 ? 1 : P.ns_area);
        cur = (cur & 0xffu) | ((uint32_t)ls << 8) | ((uint32_t)li << 16);
        PT_STAMP(S_NEE);
        // With more light samples to take, the bounce waits for the shading
        // round after the last shadow ray.  After the last one it is sampled
        // now (every light draw precedes the BSDF draws, as in trace_ray) and
        // the lane goes on with the next extension ray -- the bounce, or the
        // next sample's camera ray -- where the shadow ray ends, inside the
        // traversal loop: one shading round per path vertex, not two.
        if (emitted && !emit_last) {
          shadow = SH_RESUME;
          mode = M_TRAV;
        } else if ((int)(cur & 0xffu) >= P.max_depth) {
          finish = true;
          after = emitted;
        } else {
          // ---- indirect bounce (pathtracer.cpp:527-552)
          float3 wi;
          float pdf = 1.0f;
          float3 f;
          if (btype == 0 || btype == 4) {  // cosine hemisphere (sampler.cpp:44-55)
            float r1 = PT_DRAW();
            float r2 = PT_DRAW();
            float ct = fsqrt(1.0f - r1);  // cos(acos(1 - 2 r1) / 2)
            float stt = fsqrt(r1);
            wi = f3(stt * cos_rev(r2), stt * sin_rev(r2), ct);  // phi = 2 pi r2
            pdf = ct * 0.31830988618379067f;
            f = btype == 0 ? PT_BSDF3(bsdf, a) * 0.31830988618379067f : f3(0, 0, 0);
          } else if (btype == 1) {  // MirrorBSDF::sample_f (bsdf.cpp:60-69)
            // w_out (pathtracer.cpp:449-453) is only read by mirror / glass
            // sampling, which never waits for a shadow ray (f() = 0 there):
            // tr still holds the incoming ray, so it is rebuilt here, not kept.
            const float3 wo = normalize(fr.to_local(f3(0, 0, 0) - tdir(tr)));
            wi = f3(-wo.x, -wo.y, wo.z);
            f = PT_BSDF3(bsdf, a) * (1.0f / fmaxf(wo.z, 1e-8f));
          } else {  // Refraction (bsdf.cpp:90-111) / Glass (bsdf.cpp:120-158)
            const float3 wo = normalize(fr.to_local(f3(0, 0, 0) - tdir(tr)));
            float ratio = bsdf_f(bsdf, offsetof(DBsdf, ior) / 4);
            float sgn = 1.0f;
            if (wo.z > 0.0f) {
              sgn = -1.0f;
              ratio = 1.0f / ratio;
            }
            float cos2 = 1.0f - ratio * ratio * (1.0f - wo.z * wo.z);
            bool tir = cos2 < 0.0f;
            wi = tir ? f3(-wo.x, -wo.y, wo.z) : normalize(f3(-wo.x * ratio, -wo.y * ratio, sgn * fsqrt(cos2)));
            float ni = bsdf_f(bsdf, offsetof(DBsdf, ior) / 4), no = 1.0f;
            if (wo.z < 0.0f) {
              ni = 1.0f;
              no = bsdf_f(bsdf, offsetof(DBsdf, ior) / 4);
            }
            float inv_cos = 1.0f / fmaxf(fabsf(wi.z), 1e-8f);
            if (btype == 2) {
              f = tir ? f3(0, 0, 0) : PT_BSDF3(bsdf, t) * ((no / ni) * (no / ni) * inv_cos);
            } else if (tir) {
              f = PT_BSDF3(bsdf, t) * inv_cos;  // quirk kept: TIR returns transmittance (bsdf.cpp:129-131)
            } else {
              float ci = fabsf(wi.z), co = fabsf(wo.z);
              float r1 = (no * ci - ni * co) / (no * ci + ni * co);
              float r2 = (ni * ci - no * co) / (ni * ci + no * co);
              float Fr = 0.5f * (r1 * r1 + r2 * r2);
              if (PT_DRAW() <= Fr) {
                wi = f3(-wo.x, -wo.y, wo.z);
                f = PT_BSDF3(bsdf, a) * (1.0f / fmaxf(fabsf(wi.z), 1e-8f));
              } else {
                f = PT_BSDF3(bsdf, t) * ((no / ni) * (no / ni) * inv_cos);
              }
            }
          }
          // Russian roulette (pathtracer.cpp:534-541)
          float pterm = fmaxf(1.0f - illum(f), 0.0f);
          if (PT_DRAW() < pterm) {
            if (DBG && pix_index(pix) == P.dbg_pix) printf("    RR terminate (p=%.4g)\n", pterm);
            finish = true;
            after = emitted;
          } else {
            if (DBG && pix_index(pix) == P.dbg_pix) printf("    bounce wi=(%.6g %.6g %.6g) pdf %.5g p %.4g dim word %08x\n", wi.x, wi.y, wi.z, pdf, pterm, rdim);
            T = mul(T, f * (fabsf(wi.z) * rcp(pdf * (1.0f - pterm))));
            float3 v = normalize(fr.to_world(wi));
            const float3 bo = offset_ray(hp, dot(v, ng) >= 0.0f ? ng : f3(0, 0, 0) - ng);
            if (emitted) {  // (only Diffuse emits shadow rays, so tr.d above was never read)
              hp = bo;      // the bounce ray waits in (hp, ns) behind the shadow ray in tr
              ns = v;
              shadow = SH_FOLLOW;
            } else {
              trav_init(tr, bo, v, 3.0e38f, false);
              shadow = 0;
            }
            mode = M_TRAV;
            includeLe = btype == 1 || btype == 2 || btype == 3;
            ++cur;  // depth + 1
            if (STATS) n_bounce++;
          }
        }
      }
      if (finish) {
        ++sample;
        if (!group_ends(sample)) {
          mode = M_CAMERA;  // after a shadow ray: the camera ray goes to (hp, ns), behind it
          if (after) shadow = SH_FOLLOW;
        } else if (after) {  // refill in this round; the one store waits for the shadow ray
          PT_FENCE3(pend);  // (no contraction into pend's last multiply: the sum rounds as at the shadow ray's return)
          pend = acc + pend;
          oslot = myslot;
          ng = f3(0, 0, 0);  // (the next group's sum while the store is pending)
          PT_SLOT_DONE();
          shadow = SH_STORE;
          mode = M_FETCH;
        } else {
          group_end = true;
        }
      }
      if (group_end) {
        store_sum(P.partial + 3 * (size_t)myslot, acc);
        PT_SLOT_DONE();
        mode = M_FETCH;
      }
      PT_STAMP(S_BSDF);
    }
    // ---- refill: wave-aggregated pixel fetch (one atomic per wave per round)
    // and camera rays.  Camera rays that miss the scene's root box carry zero
    // radiance (no environment light, pathtracer.cpp:421-426): they are
    // completed here without touching memory, so background pixels never
    // occupy a traversal slot.
    for (;;) {
      bool need = mode == M_FETCH;
      unsigned long long m = __ballot(need);
      if (m != 0ull) {
        // Lanes are served from the wave's private chunk of P.chunk
        // consecutive slots; one atomic on a queue head (memory-side, since
        // the XCD L2s are not coherent; PT_QUEUE_HEADS of them, a wave starting
        // at its XCD's) refills it.  The claim size (128 / 256 / 512) and the
        // heads' dealing (interleaved chunks or contiguous bands) are chosen
        // on the host per launch (pt_api.cpp launch; profiles/r5/ab_chunk_*.txt,
        // ab_queue_heads.txt, ab_bands*.txt).
        uint32_t cnt = (uint32_t)__popcll(m);
        uint32_t avail = chunk_end - chunk_next;
        uint32_t nbase = 0, csize = 0;
        if (cnt > avail) {
          if (seen >= total_slots) {
            // This wave already saw the queue drained: every further claim
            // would fail.  No atomic -- in the drain, one per wave per round
            // on the single queue head (memory-side, serialised, slower from
            // the XCDs far from its channel) stalled every round of the
            // remaining paths (C3: the XCDs' median drain 380 vs 680 us).
            nbase = total_slots;
          } else if (first_claim) {
            // The wave's first chunk is dealt statically (chunk wave_id): at
            // the launch's start every wave would otherwise queue on the one
            // head at once (memory-side atomics, serialised), and the last
            // ones would wait for thousands of others before their first ray.
            csize = (uint32_t)P.chunk;
            nbase = wave_id * csize;
            seen = nbase + csize;
            first_claim = false;
          } else {
            csize = (uint32_t)P.chunk;
#if PT_CENSUS
            const unsigned long long c_t0 = census ? wall_clock64() : 0ull;
#endif
            const uint32_t base0 = n_waves * csize;  // (after the statically dealt chunks)
            // PT_QUEUE_HEADS heads, one per XCD, each in its own 128-B line:
            // head h deals chunks h, h + H, h + 2H, ... -- the same interleaved
            // sweep of the frame as one head, with 1/H of the atomics on each
            // line.  A wave whose head ran dry moves on to the next one.
            nbase = total_slots;
            for (int t = 0; t < PT_QUEUE_HEADS; ++t) {  // (wave-uniform; one pass but at the very end)
              uint32_t r = 0;
              if (lane == 0) r = atomicAdd(P.work_counter + qh * PT_QUEUE_WORDS, 1u);
              r = __builtin_amdgcn_readfirstlane(__shfl(r, 0));
              uint64_t cand;
              if (P.qbands) {  // (wave-uniform)
                // head h deals the h-th of H contiguous bands of the dynamic
                // slots: an XCD's waves render neighbouring pixels, whose rays
                // share BVH nodes in that XCD's L2 (host: large frames only)
                const uint32_t span = total_slots > base0 ? total_slots - base0 : 0u;
                const uint32_t band = (span + PT_QUEUE_HEADS * csize - 1u) / (PT_QUEUE_HEADS * csize) * csize;
                cand = (uint64_t)r * csize < (uint64_t)band ? (uint64_t)base0 + (uint64_t)qh * band + (uint64_t)r * csize
                                                           : (uint64_t)total_slots;
              } else {  // interleaved: head h deals chunks h, h + H, ...
                cand = (uint64_t)base0 + ((uint64_t)r * PT_QUEUE_HEADS + qh) * csize;
              }
              if (cand < (uint64_t)total_slots) {
                nbase = (uint32_t)cand;
                break;
              }
              qh = (qh + 1u) % PT_QUEUE_HEADS;
            }
            if (nbase >= total_slots) csize = 0;  // every head ran dry: drained
#if PT_CENSUS
            if (census) {  // (diagnostics: how long the claim's atomics took to return)
              asm volatile("" ::"s"(nbase));
              const unsigned long long c_d = wall_clock64() - c_t0;
              census_claim += c_d;
              census_claim_max = c_d > census_claim_max ? c_d : census_claim_max;
              ++census_claims;
            }
#endif
            seen = nbase + csize;
            // (several heads: the end of one head's range -- the last chunk of
            // the frame, or of a band -- is not the queue's; the wave has seen
            // the queue drained only when every head was dry, csize == 0)
            if (csize != 0u) seen = min(seen, total_slots - 1u);
            if (STATS) n_atomics += lane == 0;
          }
        }
        // Work slots -> (block k, pixel q, group j): see KParams (a fastdiv)
        // (MF: the slot within its frame; a frame's slots are a multiple of
        // 64 * n_groups, so no chunk of a block-aligned claim straddles two)
        auto local_slot = [&](uint32_t slot) -> uint32_t {
          if constexpr (MF) return slot - pt_fastdiv(slot, P.frm_m, P.frm_sh) * P.frame_slots;
          else return slot;
        };
        auto decode = [&](uint32_t slot, uint32_t& k, uint32_t& j, uint32_t& q) {
          slot = local_slot(slot);
          const uint32_t px = pt_fastdiv(slot, P.grp_m, P.grp_sh);
          j = slot - px * (uint32_t)P.n_groups;
          k = px >> 6;
          q = px & 63u;
        };
        auto block_of = [&](uint32_t slot) -> uint32_t { return pt_fastdiv(local_slot(slot), P.grp_m, P.grp_sh) >> 6; };
        // A chunk of 128 slots (128-aligned) lies inside one block when a
        // pixel has an even number of groups, and the lanes are
        // served from at most two chunks -- the rest of the old one and the
        // new one: both block records are read through the scalar cache
        // (wave-uniform addresses) instead of one vector-memory load per lane,
        // which every refill round would wait on (C5 +1%, framed C3 +0.3%,
        // C3 neutral: profiles/r3/ab_scalar_blocks.txt).
        const bool sblocks = P.sblocks && total_slots > 0u;  // (no blocks: nothing to read)
        int4 b_old = make_int4(0, 0, 0, 0), b_new = make_int4(0, 0, 0, 0);
        uint32_t k_old = 0, k_new = 0;
        if (sblocks) {
          typedef __attribute__((address_space(4))) const pt_v4i cst_v4i;
          const cst_v4i* cb = (const cst_v4i*)P.blocks;
          if (avail > 0u) {
            k_old = block_of(min(chunk_next, total_slots - 1u));
            const pt_v4i v = cb[k_old];
            b_old = make_int4(v.x, v.y, v.z, v.w);
          }
          if (cnt > avail) {
            k_new = block_of(min(nbase, total_slots - 1u));
            const pt_v4i v = cb[k_new];
            b_new = make_int4(v.x, v.y, v.z, v.w);
          }
        }
        if (need) {
          uint32_t rank = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
          uint32_t slot = rank < avail ? chunk_next + rank : nbase + (rank - avail);
          if (slot >= total_slots) {
            // past the end of the claimed chunk's range: retire once the queue
            // is drained; otherwise (a partial last chunk of one head's range)
            // stay M_FETCH for the refill's next claim
            if (seen >= total_slots) {
              mode = shadow ? M_TRAV : M_DONE;  // (a pending shadow ray is traced first)
              if ((STATS || (PT_CENSUS && census)) && w_empty == 0ull) w_empty = wall_clock64();
            }
          } else {
            // Blocks are <= 8x8 pixel rectangles of the tiles, clipped to the
            // scene's screen footprint (pixels outside are written 0 by
            // resolve_kernel: every ray through them misses the root box).
            uint32_t k, j, q;
            decode(slot, k, j, q);  // (the scalar path's k is the same)
            int4 b;  // (odd group counts: one vector-memory load per lane)
            if (sblocks) b = rank < avail ? b_old : b_new;
            else b = P.blocks[k];
            const int qx = (int)(q & 7u), qy = (int)(q >> 3);
            if (qx < b.z && qy < b.w) {
              pix = (b.x + qx) | ((b.y + qy) << 16);
              sample = (int)j * P.group_spp;
              myslot = slot;
              if (!shadow) acc = f3(0, 0, 0);
              else ng = f3(0, 0, 0);  // (SH_STORE: acc holds the last group's total until its store)
              if (STATS) slot_t0 = wall_clock64();
              mode = M_CAMERA;
            }
          }
        }
        if (cnt > avail) {  // wave-uniform
          chunk_end = min(nbase + csize, total_slots);  // (a partial last chunk ends at the frame's end)
          chunk_next = min(nbase + (cnt - avail), chunk_end);
          if (csize == 0) chunk_next = chunk_end = total_slots;  // drained: nothing left to hand out
        } else {
          chunk_next += cnt;
        }
      }
      PT_STAMP(S_FETCH);
      // ---- camera rays: Camera::generate_ray (camera.cpp:113-129) at the
      // jittered pixel position of raytrace_pixel (pathtracer.cpp:571-575)
      // A lane whose shadow ray is still to be traced (shadow != 0: the
      // sample ended with its last light sample) keeps that ray in tr and
      // parks the camera ray in (hp, ns), to start when the shadow ray ends.
      while (mode == M_CAMERA) {
        Trav cr;
        float3 cd;
        const bool in = camera_ray(cr, cd);
        if (!shadow) tr = cr;
        if (in) {
          T = f3(1, 1, 1);
          cur = 0;  // depth 0
          includeLe = true;
          if (shadow) {
            hp = cr.o;
            ns = cd;
            if (shadow == SH_STORE) shadow = SH_STORE_FOLLOW;
          }
          mode = M_TRAV;
          break;
        }
        // miss: the sample sees the environment (includeLe) or nothing.  With
        // a store pending (SH_STORE) acc still holds the last group's total:
        // the new group's sum gathers in ng, dead until the next hit record.
        // (Behind a pending light sample of the SAME group, SH_FOLLOW, the
        // map's radiance is added before that sample: (acc + env) + pend
        // where trace_ray's order is (acc + pend) + env -- one reordered
        // float addition at silhouettes against the map, inside the
        // near-exact tolerance; parking such rays instead cost C5 18%.)
        if (ENV) {
          const float3 e = env_dir(P, cd);
          if (shadow == SH_STORE) ng = ng + e;
          else acc = acc + e;
        }
        ++sample;
        if (group_ends(sample)) {
          if (shadow == SH_FOLLOW) {  // the pending light sample belongs to this group: one store, deferred
            PT_FENCE3(pend);  // (no contraction into pend's last multiply: the sum rounds as at the shadow ray's return)
            pend = acc + pend;
            oslot = myslot;
            ng = f3(0, 0, 0);  // (the next group's sum while the store is pending)
            shadow = SH_STORE;
          } else {  // SH_STORE: this group's sum is in ng (acc holds the last group's)
            store_sum(P.partial + 3 * (size_t)myslot, shadow ? ng : acc);
          }
          PT_SLOT_DONE();
          mode = M_FETCH;
        }
      }
      PT_STAMP(S_CAMERA);
      if (__ballot(mode == M_FETCH) == 0ull) break;
    }
    // Drain helpers: once the wave's share of the queue is gone, its retired
    // lanes (M_DONE) take the shadow rays just emitted by lanes with an
    // extension ray behind them (SH_FOLLOW), and those lanes start that ray
    // at once instead of after the shadow ray: the two rays of a path vertex
    // are traced side by side, which shortens the paths the launch ends on.
    // The k-th such lane is paired with the k-th retired one through two
    // cross-lane permutes; the helper copies the ray (o, d, 1/d, tmax), and
    // the owner applies the result when its helper is done (above).
    if constexpr (!DBG && !BIN) {
      const unsigned long long idle = __ballot(mode == M_DONE);
      const bool want = mode == M_TRAV && shadow == SH_FOLLOW && tr.node == 0;
      const unsigned long long wm = __ballot(want);
      if (P.helpers && idle != 0ull && wm != 0ull) {  // (wave-uniform)
        const unsigned long long lt = (1ull << lane) - 1ull;
        const int ri = __popcll(idle & lt), rw = __popcll(wm & lt);
        const int np = min(__popcll(idle), __popcll(wm));
        // lane r of idl / own: the lane of the r-th retired / wanting lane
        // (the others write to lane 63, which no pair reads: the two sets are
        // disjoint, so both are non-empty only with fewer than 64 members each)
        const int idl = __builtin_amdgcn_ds_permute((mode == M_DONE ? ri : 63) << 2, lane);
        const int own = __builtin_amdgcn_ds_permute((want ? rw : 63) << 2, lane);
        const bool helper = mode == M_DONE && ri < np;
        const bool owner = want && rw < np;
        const int o_lane = __builtin_amdgcn_ds_bpermute(min(ri, 63) << 2, own);
        const int h_lane = __builtin_amdgcn_ds_bpermute(min(rw, 63) << 2, idl);
        const int src = (helper ? o_lane : lane) << 2;
        auto pull = [&](float v) { return __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(v))); };
        const float3 so = f3(pull(tr.o.x), pull(tr.o.y), pull(tr.o.z));
        const float3 si = f3(pull(tr.inv.x), pull(tr.inv.y), pull(tr.inv.z));
        const float3 sd = f3(pull(tr.d.x), pull(tr.d.y), pull(tr.d.z));
        const float st = pull(tr.tmax);
        if (helper) {
          tr.o = so;
          tr.d = sd;
          tr.inv = si;
          tr.tmax = st;
          tr.node = 0;
          tr.sp = 0;
          tr.any = true;
          tr.found = false;
          tr.prim = -1;
          mode = M_TRAV;
          shadow = SH_HELPER;
        }
        if (owner) {
          trav_init(tr, hp, ns, 3.0e38f, false);
          shadow = 0;
          hl = h_lane;
        }
      }
    }
    // ================= traversal phase =================
    __builtin_amdgcn_s_setprio(PT_PRIO_TRAV);
    // Step every in-flight ray one node at a time; leave as soon as `batch`
    // lanes have finished their ray, so finished lanes are refilled together
    // (coherent shading) while the others keep their traversal state.
    if (__ballot(mode == M_TRAV) == 0ull) break;  // every lane is M_DONE
    // (Pinning the loop's parameters in SGPRs for the phase through an empty
    // asm -- so the re-read parameters are not re-loaded per iteration --
    // measured C5 -2.5%, C3 -3%: the scalar loads hide behind the node
    // step's vector loads; profiles/r4/ab_layout.txt)
    const DNode* t_nodes = P.nodes;
    const DPrim* t_prims = P.prims;
    const int t_leaf_weight = P.leaf_weight;
    // Fresh rays (node 0: references only point forward, so no ray returns
    // to the root) take their root step here, all together, from the LDS
    // copy: the wave's first traversal iteration no longer waits on a global
    // load for them.
    if constexpr (!BIN) {
      bool done = false;
      if (mode == M_TRAV && tr.node == 0) {
        done = node_step<STATS, true>(t_nodes, stk, tr, ct, (lds_cchar*)s_root);
        if (done) mode = M_SHADE;
      }
      follow_on(done);  // (a shadow ray leaves the root only if it misses every child box)
    }
    // Once the queue is drained, lanes retire (M_DONE): shade when 3/4 of the
    // lanes still working are ready, not when `batch` of 64 are, or the tail
    // would wait for the slowest ray of the wave at every bounce.
    const int alive = __popcll(__ballot(mode != M_DONE));
#if PT_CENSUS
    if (census && seen >= total_slots) {  // (diagnostics: the wave's drain)
      if (census_alive < 0) census_alive = alive;
      ++census_rounds;
    }
#endif
    int round_batch = min(batch, (3 * alive + 3) / 4);
    if (P.drain_div > 0 && seen >= total_slots)  // the queue is drained: latency, not throughput
      round_batch = max(1, alive / P.drain_div);
    if (STATS) n_rounds += lane == 0;
    if (STATS) n_rounds_drain += lane == 0 && seen >= total_slots;
    if (STATS) r_rounds += mode == M_TRAV;
    for (;;) {
      if (STATS) n_titer += lane == 0;
      if (STATS) n_titer_drain += lane == 0 && seen >= total_slots;
      // one kind of step per iteration: leaf steps once enough lanes wait on
      // a leaf (or nothing else is left), node steps otherwise
      const bool trav = mode == M_TRAV;
      const bool at_leaf = trav && tr.node < 0;
      // ballots of single compares, combined in SGPRs: a ballot of a combined
      // condition is re-materialised through a VGPR (v_cndmask + v_cmp) by the
      // compiler, twice per iteration (C3 +2.5%: profiles/r5/ab_order_ballot.txt)
      const unsigned long long b_trav = __ballot(mode == M_TRAV), b_leaf = __ballot(tr.node < 0);
      const int n_leaf = __popcll(b_trav & b_leaf);
      const int n_node = __popcll(b_trav & ~b_leaf);
      bool done = false;
      // (n_leaf > 0 and n_node == 0 need no tests of their own: some lane
      // traverses, so n_leaf * w >= n_node * 16 is false for n_leaf == 0 and
      // true for n_node == 0 -- two scalar compare-and-branches fewer)
      const bool leaf_iter = n_leaf * t_leaf_weight >= n_node * 16;
      if (STATS && trav) {
        const bool stepped = leaf_iter == at_leaf;
        r_steps += stepped;
        r_idle += !stepped;
      }
      if (STATS && !BIN) {  // node-step census (wave-uniform values)
        const bool ns = trav && !at_leaf && !leaf_iter;
        const unsigned long long nm = __ballot(ns);
        if (nm != 0ull) {
          const int fnode = __shfl(tr.node, __ffsll((long long)nm) - 1);
          const unsigned long long same = __ballot(ns && tr.node == fnode);
          const unsigned long long t2 = __ballot(ns && (uint32_t)tr.node < 21u);
          const unsigned long long t3 = __ballot(ns && (uint32_t)tr.node < 85u);
          ++c_wsteps;
          c_uniform += same == nm;
          c_cover += (uint32_t)__popcll(same);
          c_lanes += (uint32_t)__popcll(nm);
          c_top2w += t2 == nm;
          c_top2l += (uint32_t)__popcll(t2);
          c_top3w += t3 == nm;
          c_top3l += (uint32_t)__popcll(t3);
        }
      }
      if (STATS) {  // what each lane does in this iteration (SIMD efficiency)
        l_other += trav && leaf_iter != at_leaf;
        l_ready += mode == M_SHADE;
        l_dead += mode == M_DONE;
        l_leaf += at_leaf && leaf_iter;
        l_deep += trav && tr.sp > PT_STACK;
      }
      // (if / else-if: two independent ifs -- a leaf-step block and a
      // node-step block, as a both-kinds drain mode needs -- measured C3 -2%,
      // and stepping both kinds once the queue is drained did not win it back:
      // profiles/r4/ab_bisect_2.txt)
      if (leaf_iter) {
        if (at_leaf) done = leaf_step<STATS, TRI>(t_prims, stk, tr, ct);
        if (STATS) n_leafit += lane == 0;
      } else if (trav && !at_leaf) {
        if constexpr (BIN) done = node_step2<STATS>(P.nodes2, stk, tr, ct);
        else done = node_step<STATS>(t_nodes, stk, tr, ct);
      }
      if (done) mode = M_SHADE;
      follow_on(done);
      if (STATS && done) {
        ray_steps_max = max(ray_steps_max, r_steps);
        ray_idle_max = max(ray_idle_max, r_idle);
        ray_rounds_max = max(ray_rounds_max, r_rounds);
        r_steps = r_idle = r_rounds = 0;
      }
      unsigned long long ready = __ballot(mode == M_SHADE);
      unsigned long long busy = __ballot(mode == M_TRAV);
      if (busy == 0ull || __popcll(ready) >= round_batch) break;
    }
    PT_STAMP(S_TRAV);
  }

  if (census && lane == 0) census[2] = wall_clock64();
#if PT_CENSUS
  if (census) {
    // first time a lane of the wave found the queue empty, its lanes alive
    // then, the wave's rounds from then on
    unsigned long long e = w_empty ? w_empty : ~0ull;
    for (int off = 32; off > 0; off >>= 1) {
      const unsigned long long o = __shfl_xor(e, off);
      e = o < e ? o : e;
    }
    if (lane == 0) {
      census[1] = e;
      census[4] = (unsigned long long)census_alive;
      census[5] = (unsigned long long)census_rounds;
      census[6] = census_claim;
      census[7] = census_claims;
      census[8] = census_claim_max;
    }
  }
#endif
  if (STATS) {
    PT_STAMP(S_OTHER);
    unsigned long long v[11] = {n_cam, n_bounce, n_shadow, ct.nodes, ct.tris, ct.spheres, n_hits,
                                n_titer, n_rounds, n_leafit, n_atomics};
    for (int k = 0; k < 11; ++k) {
      unsigned long long s = v[k];
      for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off);
      if (lane == 0) atomicAdd(P.stats + k, s);
    }
    if (lane < 32) atomicAdd(P.stats + 32 + lane, (unsigned long long)s_hist[lane]);
    const uint32_t li[5] = {l_other, l_ready, l_dead, l_leaf, l_deep};
    for (int k = 0; k < 5; ++k) {
      unsigned long long s = li[k];
      for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off);
      if (lane == 0) atomicAdd(P.stats + 27 + k, s);
    }
    // load balance: the slowest wave bounds the launch
    w_empty = w_empty ? w_empty : ~0ull;
    for (int off = 32; off > 0; off >>= 1) {
      const unsigned long long o = __shfl_xor(w_empty, off);
      w_empty = o < w_empty ? o : w_empty;
    }
    uint32_t slots_done = n_cam;  // camera samples this wave started
    for (int off = 32; off > 0; off >>= 1) {
      slots_done += __shfl_xor(slots_done, off);
      slot_lat_sum += __shfl_xor(slot_lat_sum, off);
      const unsigned long long o = __shfl_xor(slot_lat_max, off);
      slot_lat_max = o > slot_lat_max ? o : slot_lat_max;
      ray_steps_max = max(ray_steps_max, (uint32_t)__shfl_xor((int)ray_steps_max, off));
      ray_idle_max = max(ray_idle_max, (uint32_t)__shfl_xor((int)ray_idle_max, off));
      ray_rounds_max = max(ray_rounds_max, (uint32_t)__shfl_xor((int)ray_rounds_max, off));
    }
    if (lane == 0) {
      // wave clocks: every section of the wave's lifetime, traversal apart
      const unsigned long long trav = s_clk[S_TRAV];
      const unsigned long long hitshade = s_clk[S_HIT] + s_clk[S_NEE] + s_clk[S_BSDF];
      const unsigned long long shade = hitshade + s_clk[S_FETCH] + s_clk[S_CAMERA] + s_clk[S_OTHER];
      atomicAdd(P.stats + 11, shade);
      atomicAdd(P.stats + 12, trav);
      atomicMax(P.stats + 13, shade + trav);
      atomicAdd(P.stats + 16, hitshade);
      for (int k = 0; k < 4; ++k) atomicAdd(P.stats + 17 + k, s_clk[S_HIT + k]);
      unsigned long long w = wall_clock64() - w_start;
      const unsigned long long w_end = wall_clock64();  // launch shape: first/last wave start and end
      atomicMin(P.stats + 21, w_start);
      atomicMax(P.stats + 22, w_start);
      atomicMin(P.stats + 23, w_end);
      atomicMax(P.stats + 24, w_end);
      if (w_empty != ~0ull) {
        atomicMin(P.stats + 25, w_empty);
        atomicMax(P.stats + 26, w_empty);
      }
      atomicAdd(P.stats + 14, w);
      atomicMax(P.stats + 15, w);
      const uint32_t cn[8] = {c_wsteps, c_uniform, c_cover, c_lanes, c_top2w, c_top2l, c_top3w, c_top3l};
      for (int k = 0; k < 8; ++k) atomicAdd(P.stats + 64 + k, (unsigned long long)cn[k]);
      // per-wave trace (pt_get_wave_trace): start, first empty queue, end,
      // (XCC id << 32 | HW_ID), camera samples
      unsigned long long* tw = P.stats + PT_STATS_SLOTS + PT_WAVE_TRACE * (size_t)wave_id;
      tw[0] = w_start;
      tw[1] = w_empty;
      tw[2] = w_end;
      tw[3] = ((unsigned long long)__builtin_amdgcn_s_getreg((3 << 11) | 20) << 32) |
              (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
      tw[4] = slots_done;
      tw[5] = slot_lat_sum;
      tw[6] = slot_lat_max;
      tw[7] = ((unsigned long long)ray_steps_max << 32) | ray_idle_max;
      tw[8] = ray_rounds_max;
      tw[9] = n_titer_drain;
      tw[10] = n_rounds_drain;
    }
  }
}

#undef P

#if !PT_ENV_TU  // (pt_kernels_env.hip emits only the ENV render kernels)
// Sums each pixel's sample groups in group order, so the sum is a fixed
// function of the pixel, independent of scheduling and of the tile -> GPU
// assignment, and writes the pixel's average, SampleBuffer-style
// (pathtracer.cpp:577-581).  One workgroup per tile: the tile's pixels outside
// the scene's screen footprint are written 0; then its blocks, four at a time,
// one lane per pixel: a block's 64 pixels' group sums are one contiguous run
// of 64 * n_groups * 12 B (pixel-major).
__global__ __launch_bounds__(256) void resolve_kernel(KParams P) {
  const int ti = (int)blockIdx.x;
  const int4 tile = P.tiles[ti];
  const int tid = (int)threadIdx.x;
  // the render that wrote these sums is complete, so are its queue claims:
  // zero the heads for the render slot's next launch (pt_api.cpp launch)
  if (ti == 0)
    for (int i = tid; i < PT_QUEUE_WORDS * PT_QUEUE_HEADS; i += 256) P.work_counter[i] = 0u;
  auto out_at = [&](int x, int y) -> float* {
    const size_t ps = (size_t)P.packed;  // packed slot edge (32, or 16 with PT_FLAG_PACKED16); 0: the frame
    const size_t oi = P.tile_out ? (size_t)P.tile_out[ti] : (size_t)ti;  // (the caller's tile index)
    const size_t o = ps ? oi * ps * ps + (size_t)(y - tile.y) * ps + (size_t)(x - tile.x)
                        : (size_t)x + (size_t)y * (size_t)P.W;
    return P.out + 3 * o;
  };
  for (int i = tid; i < 1024; i += 256) {
    const int x = tile.x + (i & 31), y = tile.y + (i >> 5);
    if ((i & 31) < tile.z && (i >> 5) < tile.w && culled(P, x, y)) store3(out_at(x, y), f3(0, 0, 0));
  }
  const float inv_spp = (float)(1.0 / (double)P.spp);
  const int q = tid & 63, qx = q & 7, qy = q >> 3;
  const int b1 = P.tile_block0[ti + 1];
  for (int k = P.tile_block0[ti] + (tid >> 6); k < b1; k += 4) {
    const int4 b = P.blocks[k];
    if (qx >= b.z || qy >= b.w) continue;
    float3 acc = f3(0, 0, 0);
    const float* pa = P.partial + 3 * ((size_t)k * 64u + (size_t)q) * (size_t)P.n_groups;
    if ((P.n_groups & 3) == 0) {
      // The pixel's run of n_groups 12-B sums (16-B aligned: 48 B per four
      // groups) read as 16-B vectors, four groups (three loads) per step: a
      // wave's 64 runs lie 12 * n_groups B apart, and with one 12-B load per
      // group every load instruction touched 64 lines that the L1 had evicted
      // again before the next group's load came (lone resolve C3 0.047 ->
      // 0.033 ms, C4 0.36 -> 0.23 ms).  Same summation order (group 0, 1,
      // 2, ...).  At most 24 VGPRs: the resolve runs beside the next frame's
      // render waves (5 per SIMD at <= 96 VGPRs leave 32 per SIMD); with 40
      // it waited for them (pipelined C3 -5%: profiles/r5/ab_resolve_wide.txt).
      const float4* pv = (const float4*)pa;
#pragma unroll 1
      for (int j = 0; j < P.n_groups; j += 4, pv += 3) {
        float4 v[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) v[i] = pv[i];
        const float* f = &v[0].x;
#pragma unroll
        for (int g = 0; g < 4; ++g) acc = acc + f3(f[3 * g], f[3 * g + 1], f[3 * g + 2]);
      }
    } else {
#pragma unroll 2
      for (int j = 0; j < P.n_groups; ++j) acc = acc + ld3(pa + 3 * (size_t)j);
    }
    store3(out_at(b.x + qx, b.y + qy), acc * inv_spp);
  }
}

// Batched BVHAccel::intersect queries, one lane per ray.
__global__ __launch_bounds__(PT_BLOCK) void intersect_kernel(const DNode* __restrict__ nodes,
                                                           const DPrim* __restrict__ prims, const float* __restrict__ o,
                                                           const float* __restrict__ d, const float* __restrict__ maxt,
                                                           int64_t n, int32_t* hit, float* t, int32_t* prim,
                                                           int32_t* anyhit, int* spill, const int* prim_map) {
  __shared__ int s_stack[PT_STACK * PT_BLOCK];
  int64_t i = (int64_t)blockIdx.x * PT_BLOCK + threadIdx.x;
  const Stack stk{(lds_int*)(s_stack + threadIdx.x), spill, gridDim.x * PT_BLOCK};
  if (i >= n) return;
  float3 O = f3(o[3 * i], o[3 * i + 1], o[3 * i + 2]);
  float3 D = f3(d[3 * i], d[3 * i + 1], d[3 * i + 2]);
  Hit h;
  h.t = 0;
  h.prim = -1;
  Counters ct = {0, 0, 0};
  bool f = traverse<false>(nodes, prims, stk, O, D, 3.0e38f, false, h, ct);
  hit[i] = f ? 1 : 0;
  t[i] = f ? h.t : -1.0f;
  prim[i] = f ? (prim_map ? prim_map[h.prim] : h.prim) : -1;
  Hit h2;
  bool a = traverse<false>(nodes, prims, stk, O, D, maxt[i], true, h2, ct);
  anyhit[i] = a ? 1 : 0;
}

#endif  // !PT_ENV_TU

}  // namespace ptk

// ------------------------------------------------------------------ launchers
template <bool ENV, bool GTAB>
static void launch_render(const KParams* P, int waves, bool stats, bool ref_counts, hipStream_t s) {
  const int grid = waves;  // one wave per workgroup
  const dim3 blk(PT_BLOCK);
  if (ref_counts)
    hipLaunchKernelGGL((ptk::render_kernel<true, false, true, ENV, GTAB>), dim3(grid), blk, 0, s, *P);
  else if (P->dbg_pix >= 0)
    hipLaunchKernelGGL((ptk::render_kernel<false, true, false, ENV, GTAB>), dim3(grid), blk, 0, s, *P);
  else if (stats && P->tri_only && !GTAB)
    hipLaunchKernelGGL((ptk::render_kernel<true, false, false, ENV, GTAB, true>), dim3(grid), blk, 0, s, *P);
  else if (stats)
    hipLaunchKernelGGL((ptk::render_kernel<true, false, false, ENV, GTAB>), dim3(grid), blk, 0, s, *P);
  else if (P->n_frames > 1) {  // a frame batch (host: the plain common build only)
    if constexpr (!ENV && !GTAB) {
      if (P->tri_only)
        hipLaunchKernelGGL((ptk::render_kernel<false, false, false, false, false, true, true>), dim3(grid), blk, 0, s, *P);
      else
        hipLaunchKernelGGL((ptk::render_kernel<false, false, false, false, false, false, true>), dim3(grid), blk, 0, s, *P);
    }
  } else if (P->tri_only && !GTAB)
    hipLaunchKernelGGL((ptk::render_kernel<false, false, false, ENV, GTAB, true>), dim3(grid), blk, 0, s, *P);
  else
    hipLaunchKernelGGL((ptk::render_kernel<false, false, false, ENV, GTAB>), dim3(grid), blk, 0, s, *P);
}

#if PT_ENV_TU
// Environment-light scenes: this translation unit (pt_kernels_env.hip) holds
// the ENV instantiations, built without pt_kernels.hip's scheduler option
// (build.py: iterative-ILP scheduling is +1.7% on C3, -2.9% on C5).
extern "C" hipError_t ptk_launch_render_env(const KParams* P, int grid, bool stats, bool ref_counts, bool gtab,
                                            hipStream_t s) {
  if (gtab) launch_render<true, true>(P, grid, stats, ref_counts, s);
  else launch_render<true, false>(P, grid, stats, ref_counts, s);
  return hipGetLastError();
}
extern "C" hipError_t ptk_render_occupancy_env(int* waves_per_cu, bool gtab) {
  int blocks = 0;
  hipError_t e = gtab ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                            &blocks, ptk::render_kernel<false, false, false, true, true>, PT_BLOCK, 0)
                      : hipOccupancyMaxActiveBlocksPerMultiprocessor(
                            &blocks, ptk::render_kernel<false, false, false, true, false>, PT_BLOCK, 0);
  *waves_per_cu = blocks;
  return e;
}
#else
extern "C" hipError_t ptk_launch_render_env(const KParams* P, int grid, bool stats, bool ref_counts, bool gtab,
                                            hipStream_t s);

extern "C" hipError_t ptk_launch_render(const KParams* P, int grid, bool stats, bool ref_counts, hipStream_t s) {
  static const bool force_gtab = std::getenv("PT_FORCE_GLOBAL_TABLES") != nullptr;  // tests
  const bool gtab = force_gtab || P->n_bsdfs > PT_LDS_BSDFS || P->n_lights > PT_LDS_LIGHTS;
  if (P->env_w > 0) return ptk_launch_render_env(P, grid, stats, ref_counts, gtab, s);
  if (gtab) launch_render<false, true>(P, grid, stats, ref_counts, s);
  else launch_render<false, false>(P, grid, stats, ref_counts, s);
  return hipGetLastError();
}

extern "C" hipError_t ptk_launch_resolve(const KParams* P, hipStream_t s) {
  if (P->n_tiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(ptk::resolve_kernel, dim3(P->n_tiles), dim3(256), 0, s, *P);
  return hipGetLastError();
}

extern "C" hipError_t ptk_launch_intersect(const DNode* nodes, const DPrim* prims, const float* o,
                                           const float* d, const float* maxt, int64_t n, int32_t* hit, float* t,
                                           int32_t* prim, int32_t* anyhit, int* spill, const int* prim_map,
                                           hipStream_t s) {
  int grid = (int)((n + PT_BLOCK - 1) / PT_BLOCK);
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(ptk::intersect_kernel, dim3(grid), dim3(PT_BLOCK), 0, s, nodes, prims, o, d, maxt, n,
                     hit, t, prim, anyhit, spill, prim_map);
  return hipGetLastError();
}

// Resident render waves (one-wave workgroups) per CU of the plain build of
// each variant (env, gtab) or of the STATS build of the common variant.
template <bool STATS, bool ENV, bool GTAB>
static hipError_t occupancy(int* waves_per_cu) {
  int blocks = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, ptk::render_kernel<STATS, false, false, ENV, GTAB>,
                                                              PT_BLOCK, 0);
  *waves_per_cu = blocks;
  return e;
}
extern "C" hipError_t ptk_render_occupancy_env(int* waves_per_cu, bool gtab);
extern "C" hipError_t ptk_render_occupancy(int* waves_per_cu, bool stats, bool env, bool gtab) {
  if (env) return ptk_render_occupancy_env(waves_per_cu, gtab);
  if (stats) return occupancy<true, false, false>(waves_per_cu);
  return gtab ? occupancy<false, false, true>(waves_per_cu) : occupancy<false, false, false>(waves_per_cu);
}
#endif  // PT_ENV_TU
