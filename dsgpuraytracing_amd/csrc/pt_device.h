// pt_device.h — device-side data layout of the HIP path (shared by the kernels
// and the host conversion in pt_api.cpp).  See DESIGN.md "Data layout in HBM".
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef PT_BLOCK
#define PT_BLOCK 64  // one wave64 per workgroup: the persistent queue is per wave
#endif
#ifndef PT_CHUNK
#define PT_CHUNK 128  // work slots a wave claims from the queue per atomic (KParams.chunk)
#endif
#ifndef PT_CHUNK_MAX
#define PT_CHUNK_MAX 256  // the claim for frames with >= PT_CHUNK_BIG_SLOTS slots per resident lane
#endif
#ifndef PT_CHUNK_BIG
#define PT_CHUNK_BIG 512  // the claim for large frames where it fits (pt_api.cpp launch)
#endif
#ifndef PT_BANDS_TREE_MIB
#define PT_BANDS_TREE_MIB 8  // queue bands for large frames over render trees above this size (pt_api.cpp launch)
#endif
// Frames per launch of pt_render_frames_device (KParams.seeds; include/ptgpu.h)
#ifndef PT_MAX_FRAMES
#define PT_MAX_FRAMES 8
#endif
#ifndef PT_BATCH_SLOTS
#define PT_BATCH_SLOTS 32  // a frame with more work slots per lane (of a whole MI355X) renders alone (pt_api.cpp)
#endif
#ifndef PT_SMALL_SLOTS
#define PT_SMALL_SLOTS 16  // launches with at most this many work slots per resident lane are small (pt_api.cpp launch)
#endif
#ifndef PT_CHUNK_BIG_SLOTS
#define PT_CHUNK_BIG_SLOTS 128  // C4 (184 slots per lane) +1.5%, C5 (1,620) +6.6%; C3 (26), framed C3 (51): their lone launches lose
#endif
static_assert(PT_CHUNK >= PT_BLOCK, "a refill must cover a whole wave's demand");
#define PT_QUEUE_WORDS 32  // a work-queue head, alone in its 128-B line
// Queue heads, interleaved chunk by chunk, a wave starting at its XCD's: with
// the drain helpers, 8 measured C3 +1.9% pipelined, lone launch -4.0%, C5
// +2.2%, C4 +-0 over one head (profiles/r5/ab_queue_heads.txt; a claim on the
// one head waited ~1 us: census_claims.txt).  The resolve zeroes a launch's
// heads for the render slot's next launch (pt_kernels.hip resolve_kernel).
// (Measured and removed: a tail of 64-slot claims from a second head, C3 -2.6%
// -- profiles/r5/ab_tail_claims.txt.)
#define PT_QUEUE_HEADS 8
#ifndef PT_GROUP_SPP
#define PT_GROUP_SPP 4  // default samples per work slot (pt_api.cpp group_size; 8 or more: C3 -4%, C5 -10%)
#endif
#ifndef PT_GROUP_SPP_ENV
#define PT_GROUP_SPP_ENV 2  // with an environment light
#endif
#ifndef PT_GROUP_REF_LANES
#define PT_GROUP_REF_LANES (256 * 20 * 64)  // the group-size rule's lanes: a whole MI355X at 20 waves per CU (device-independent)
#endif
#ifndef PT_GROUP_MIN_SLOTS
#define PT_GROUP_MIN_SLOTS 24  // groups are halved until the traced samples make this many slots per lane
#endif
// A group sum in memory: a packed float3, 12 B (16-B records measured C3
// -1.5%: profiles/r5/ab_order_ballot.txt).
#define PT_SUM_BYTES 12
#ifndef PT_GROUP_SUM_GIB
#define PT_GROUP_SUM_GIB 8  // group-sum budget per render slot (GiB): a group size that needs more doubles
#endif
// Leave traversal when this many lanes finished their ray (shade them
// together).  Scenes with an environment light shade longer per round (map
// lookups on every miss, inverse-CDF light samples) and want larger rounds:
// same-session sweep (profiles/r3/ab_shade_batch.txt) C3 / framed C3 / C4
// +1.5 / +3.4 / +5.6% at 32 vs 48, C5 -4% at 36 and best at 48.
#ifndef PT_SHADE_BATCH
#define PT_SHADE_BATCH 32
#endif
#ifndef PT_SHADE_BATCH_ENV
#define PT_SHADE_BATCH_ENV 48
#endif
#ifndef PT_LDS_BSDFS
#define PT_LDS_BSDFS 16  // material tables up to this size are staged in LDS
#endif
#ifndef PT_LDS_LIGHTS
#define PT_LDS_LIGHTS 8
#endif
// leaf steps when leaf lanes >= node lanes * 16 / leaf weight; with 32-lane
// shading rounds 10 beat 16 (C3 +1.9%, framed C3 +1.8%, C4 +1.4%); C5 (the
// environment-light build) is flat between 10 and 16 and keeps 16
// (profiles/r3/ab_leaf_weight.txt).  Round 4, with two-sample groups on C3:
// 12 over 10, C3 +0.8% and its lone launch -0.9%, C4 / framed C3 flat
// (profiles/r4/ab_knobs_batch_leaf.txt)
#ifndef PT_LEAF_WEIGHT
#define PT_LEAF_WEIGHT 12
#endif
#ifndef PT_LEAF_WEIGHT_ENV
#define PT_LEAF_WEIGHT_ENV 16
#endif
// One guide bucket k of a running-sum array a (environment-light CDFs), in
// one 32-B record so that a lower_bound whose window is short needs ONE
// memory round trip: the window [lo, hi] = [g[k-1], g[k+2]] of the guide
// table g, and the window's values w_i = a[min(lo + i, hi)] (i < 4), w4 =
// a[hi], wm = a[lo - 1] (0 at lo = 0).  Windows longer than four entries
// (hi - lo > 4) are halved on the array itself (record_lower_bound).
struct alignas(32) EnvRec {
  int lo, hi;
  float wm, w0, w1, w2, w3, w4;
};

// lower_bound of v = r * a[n-1] accelerated by a guide table g[0..G] with
// g[k] = lower_bound(a, k/G * a[n-1]) (built on the host, clamped to n-1): the
// answer lies in [g[k-1], g[k+2]] for k = floor(r*G), one bucket of slack
// either side for rounding, and a[g[k+2]] >= v; the result is exactly
// std::lower_bound's.  With PT_ENV_GUIDE buckets the window is a few entries
// where the CDF carries mass (where samples land).  Bucket k's record (EnvRec)
// holds the window and its values, so the usual short window (<= 4 entries)
// costs ONE memory round trip -- two 16-B loads of one 32-B record -- and
// lower_bound = lo + #{entries < v} (the array is sorted); the caller's
// interpolation pair (prev = a[t-1] or 0, cur = a[t]) comes from the same
// registers.  A longer window -- where the CDF is nearly flat (dim regions of
// a peaky map) or the map is wider than the guide table (w > PT_ENV_GUIDE:
// several entries per bucket) -- is halved on the array down to <= 4 entries
// (answer in [lo, lo + n]) and its five values re-read.  (Guide table, then
// window: two dependent round trips, C5 -1.9%: profiles/r4/ab_env_records.txt.)
// Host and device: pt_env_search_check (pt_api.cpp) replays it against
// std::lower_bound on the host (tests/test_env_search.py).
__host__ __device__ inline int record_lower_bound(const float* __restrict__ a, float v, float r,
                                                  const EnvRec* __restrict__ rec, int G, float& prev, float& cur) {
  int k = (int)(r * (float)G);
  k = k < 0 ? 0 : k > G - 1 ? G - 1 : k;
#if defined(__HIP_DEVICE_COMPILE__)
  // the record as two 16-B vector loads, both issued before the window test:
  // read through a 32-B struct copy, the compiler loads (lo, hi, wm) first and
  // sinks the w_i loads behind the branch -- a second dependent round trip
  // (C5 -1.5%, round 5)
  typedef float rf4 __attribute__((ext_vector_type(4)));
  const rf4 q0 = ((const rf4*)(rec + k))[0];
  rf4 q1 = ((const rf4*)(rec + k))[1];
  asm volatile("" : "+v"(q1));
  int lo = __float_as_int(q0.x);
  const int hi = __float_as_int(q0.y);
  float wm = q0.z, w0 = q0.w, w1 = q1.x, w2 = q1.y, w3 = q1.z, w4 = q1.w;
#else
  // host replay: one 32-B copy of the record.  (Bit-casting the int fields
  // out of float4 elements misread the window in host code -- clang's
  // __builtin_bit_cast of a vector element returns element 0 there -- which
  // the host replay caught.)
  EnvRec e;
  __builtin_memcpy(&e, rec + k, sizeof(EnvRec));
  int lo = e.lo;
  const int hi = e.hi;
  float wm = e.wm, w0 = e.w0, w1 = e.w1, w2 = e.w2, w3 = e.w3, w4 = e.w4;
#endif
  int n = hi - lo;
  if (n > 4) {
    while (n > 4) {
      const int half = n >> 1;
      if (a[lo + half] < v) {
        lo += half + 1;
        n -= half + 1;
      } else {
        n = half;
      }
    }
    auto at = [&](int i) { return a[i < hi ? i : hi]; };
    wm = lo > 0 ? a[lo - 1] : 0.0f;
    w0 = at(lo), w1 = at(lo + 1), w2 = at(lo + 2), w3 = at(lo + 3);
    w4 = at(lo + 4);  // (the record's w4 is a[hi] of the WHOLE window: ADVICE r4)
  }
  const int c = (int)(w0 < v) + (int)(w1 < v) + (int)(w2 < v) + (int)(w3 < v);
  cur = c == 0 ? w0 : c == 1 ? w1 : c == 2 ? w2 : c == 3 ? w3 : w4;
  prev = c == 0 ? wm : c == 1 ? w0 : c == 2 ? w1 : c == 3 ? w2 : w3;
  return lo + c;
}
// The drain fields of the census of plain launches (tools/wave_trace.py
// --census) are compiled in only with -DPT_CENSUS=1 (PT_HIPCC_FLAGS): their
// bookkeeping in the persistent loop cost C3 2% even when off
// (profiles/r4/census_drain.txt).
#ifndef PT_CENSUS
#define PT_CENSUS 0
#endif
#ifndef PT_ENV_GUIDE
#define PT_ENV_GUIDE 1024  // buckets of the environment-CDF guide tables (with the window compare: C5 +10% over 64, profiles/r3/ab_env_window_search.txt)
#endif
#define PT_STATS_SLOTS 72  // launch counters (32..63: slot-latency histogram, 64..71: node-step census); per-wave trace records (PT_WAVE_TRACE u64 each) follow
#define PT_WAVE_TRACE 11
#ifndef PT_STACK
#define PT_STACK 24  // traversal stack entries per lane in LDS (lane-contiguous)
#endif
#ifndef PT_STACK_MAX
#define PT_STACK_MAX 256  // deepest worst-case stack accepted (entries past PT_STACK spill to global memory)
#endif

// BVH4 node, 128 B (one L2 line): four child boxes in SoA form, component k
// of each float4 belongs to child k, then the four child references.
//  ref >= 0 is a node index; ref < 0 is a leaf cursor ~((first << 3) | (count - 1)):
//  primitives [first, first+count) in BVH order, count <= 8 (longer leaves
//  are split into subtrees).  Unused slots hold a box at +inf (never entered).
struct alignas(16) DNode {
  float4 lox, hix, loy, hiy, loz, hiz;
  int4 ref;
  int4 pad;
};

// (Round 5 built and measured two other render-tree encodings, removed in
// round 6 with their records kept: an 8-wide node with fp16 planes from a node
// origin, C3 -8.2%, and the 4-wide node compressed the same way to 80 B, C3
// -2.4%: profiles/r5/ab_stack_fast_w8.txt, ab_sel_spill_compress.txt.)

// Binary node of the reference topology, 64 B: both child boxes + child
// references (as DNode.ref).  Only traversed by the reference-count launch
// (PT_FLAG_REF_COUNTS), whose node visits feed SURVEY.md §8(d)'s cost model.
//  a = (c0.lo.x, c0.hi.x, c0.lo.y, c0.hi.y), b = the same for c1,
//  c = (c0.lo.z, c0.hi.z, c1.lo.z, c1.hi.z), e = (c0 ref, c1 ref, 0, 0)
struct alignas(16) DNode2 {
  float4 a, b, c;
  int4 e;
};

// Primitive, 48 B.  Triangle: v0 = (p1, meta), e1 = p2-p1, e2 = p3-p1.
// Sphere: v0 = (o, meta), e1 = (r, r*r, 0, 0).  meta = (bsdf << 1) | is_triangle.
struct alignas(16) DPrim {
  float4 v0, e1, e2;
};

struct alignas(16) DBsdf {
  int type;
  float a[3];  // albedo / reflectance
  float t[3];  // transmittance
  float e[3];  // emission
  float ior;
  float pad;
};

struct alignas(16) DLight {
  int type;
  float rad[3];
  float pos[3];
  float dir[3];
  float dimx[3];
  float dimy[3];
  float area;
  float pad[2];
};

struct KParams {
  float cam_pos[3];
  float c2w_col0[3], c2w_col1[3], c2w_col2[3];
  float cam_ax, cam_ay;  // screenW/screenDist, screenH/screenDist
  int W, H, spp, max_depth, ns_area;
  float nls_scale;     // (float)(1.0 / ns_area): an area light sample's weight (pathtracer.cpp:481)
  float inv_w, inv_h;  // 1/W, 1/H
  uint32_t seed;
  uint32_t sample_base;  // first sample index of the pass (RNG keys)
  int n_lights;
  int n_bsdfs;
  int n_tiles;     // 32x32 (or smaller) tiles: 1024 pixels each
  // Sample groups (work slots) of a pixel, a function of the frame only
  // (launch(): pt_api.cpp group_size): group j holds samples
  // [j * group_spp, min((j + 1) * group_spp, spp)).
  int group_spp;   // samples per work slot
  int group_shift;   // log2(group_spp) when a power of two, else -1 (shifts instead of divisions)
  int n_groups;    // ceil(spp / group_spp): work slots per pixel
  // Work slot / group-sum index of (block b, pixel q of the 8x8 block, group
  // j): (b * 64 + q) * n_groups + j -- a pixel's groups are consecutive, so a
  // wave's lanes hold a few pixels' groups (coherent camera rays).
  uint32_t grp_m, grp_sh;           // fastdiv by n_groups (pt_fastdiv)
  int sblocks;                      // every chunk lies in one block (64 * n_groups a multiple of chunk): scalar block loads
  int chunk;                        // slots per queue claim (PT_CHUNK or PT_CHUNK_MAX), a multiple of 64
  const int* tile_block0;           // first block of each tile (n_tiles + 1 entries), for the resolve
  const DNode* nodes;     // the render tree (BVH4)
  const DNode2* nodes2;  // the binary tree (reference-count launch only)
  const DPrim* prims;
  const float* norms;  // 9 floats per primitive (vertex normals n1,n2,n3)
  const DBsdf* bsdfs;
  const DLight* lights;
  int env_w, env_h;          // environment map size (0: no environment light)
  const float4* env_tex;     // map RGB, row 0 = +y
  const float* env_ptheta;   // EnvironmentLight::pTheta (running sums over rows)
  const float* env_pphi;     // pPhiGivenTheta (running sums within each row)
  const float* env_pdf;      // pThetaPhi
  const struct EnvRec* env_rtheta;  // bucket records of env_ptheta (PT_ENV_GUIDE)
  const struct EnvRec* env_rphi;    // bucket records of the rows of env_pphi (h x PT_ENV_GUIDE)
  const int4* tiles;  // (x, y, w, h)
  const int* tile_out;  // packed slot of launched tile i (the caller's index; null: i) -- a Z-ordered launch
  float* out;         // W*H*3, or n_tiles*1024*3 when packed
  int packed;         // packed slot edge S (PT_FLAG_PACKED: 32, PT_FLAG_PACKED16: 16; 0: the frame):
                      // tile i's pixel (x, y) -> out[3 * (i*S*S + (y-ty)*S + (x-tx))]
  float* partial;     // 3 floats per work slot: each sample group's sum, resolved into `out` in group order
  const int4* blocks;  // (x, y, w<=8, h<=8): footprint-clipped pixel blocks of the tiles
  int n_blocks;
  uint32_t* work_counter;
  unsigned long long* stats;  // counters (PT_FLAG_STATS / PT_FLAG_REF_COUNTS)
  int* stack_spill;           // traversal stack entries beyond PT_STACK (null if the BVH never needs them)
  int dbg_pix;                // diagnostic printf trace of one pixel (-1: off)
  int shade_batch;            // leave the traversal phase once this many lanes finished their ray
  int leaf_weight;            // leaf steps run when leaf_weight * leaf lanes >= 16 * node lanes
  int drain_div;              // queue drained: shade once alive/drain_div lanes are ready (0: 3/4 rule)
  int tri_only;               // every primitive is a triangle: the kernel without the sphere test
  int helpers;                // drain helpers on (PT_HELPERS; PT_NO_HELPERS turns them off per launch)
  int qbands;                 // queue heads deal contiguous bands, not interleaved chunks (large frames)
  int census;                 // plain build: record each wave's start / end / CU / drain in the trace area (PT_CENSUS)
  float root_lo[3], root_hi[3];  // scene bounds (root box, rounded outward)
  int cull_x0, cull_y0, cull_x1, cull_y1;  // pixels outside [x0,x1]x[y0,y1] see no geometry
  // Frame batch (pt_render_frames_device, the MF kernel): n_frames frames of
  // the same tiles in one launch.  Work slot g is slot g - f * frame_slots of
  // frame f = g / frame_slots; frame f keys its samples with seeds[f] and its
  // group sums follow frame f - 1's (partial + 3 * g).  One frame: unused.
  int n_frames;
  uint32_t frame_slots;
  uint32_t frm_m, frm_sh;  // fastdiv by frame_slots
  uint32_t seeds[PT_MAX_FRAMES];
};

// q = u / d for u < 2^31 and a runtime divisor d >= 1, without a division:
// q = m ? mulhi(u, m) >> sh : u >> sh (Granlund & Montgomery 1994).  For d
// a power of two m = 0; otherwise with 2^(l-1) < d < 2^l, m = ceil(2^(31+l) / d)
// < 2^32 and sh = l - 1: u*m / 2^(31+l) = u/d + u*e / (d * 2^(31+l)) with
// e = m*d - 2^(31+l) < d, and the error term stays below 1/d for u < 2^31, so
// the floor is exact (tests/test_abi.py checks it exhaustively for small d).
inline void pt_fastdiv_init(uint32_t d, uint32_t* m, uint32_t* sh) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  if ((1ull << l) == d) {
    *m = 0;
    *sh = l;
  } else {
    *m = (uint32_t)((((uint64_t)1 << (31 + l)) + d - 1) / d);
    *sh = l - 1;
  }
}
__device__ __forceinline__ uint32_t pt_fastdiv(uint32_t u, uint32_t m, uint32_t sh) {
  return m ? __umulhi(u, m) >> sh : u >> sh;
}

// GPU BVH build (lbvh.hip).  Inputs in upload order; outputs hipMalloc'd by
// the builder (the caller owns and frees them).
struct LbvhIn {
  int n;
  const DPrim* prims;    // device, input order
  const float* norms;    // device, 9 per primitive
  float scene_min[3], scene_extent[3];  // scene box (rounded outward)
};
struct LbvhOut {
  DPrim* prims;          // sorted order
  float* norms;
  int* prim_map;         // sorted index -> input index
  DNode* nodes4;
  int n4;
  DNode2* nodes2;
  int n2;
  int max_stack;         // worst-case traversal stack of nodes4
  float root_lo[3], root_hi[3];
};
extern "C" hipError_t ptk_build_lbvh(const LbvhIn* in, LbvhOut* out, hipStream_t s);

extern "C" hipError_t ptk_launch_render(const KParams* P, int grid, bool stats, bool ref_counts, hipStream_t s);
extern "C" hipError_t ptk_launch_resolve(const KParams* P, hipStream_t s);
extern "C" hipError_t ptk_launch_intersect(const DNode* nodes, const DPrim* prims, const float* o, const float* d,
                                           const float* maxt, int64_t n, int32_t* hit, float* t, int32_t* prim,
                                           int32_t* anyhit, int* spill, const int* prim_map, hipStream_t s);
extern "C" hipError_t ptk_render_occupancy(int* waves_per_cu, bool stats, bool env, bool gtab);
