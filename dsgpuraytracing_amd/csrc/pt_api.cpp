// pt_api.cpp — C ABI of the HIP path (include/ptgpu.h): device context, scene
// upload (reference BVH -> 64-B two-child-box nodes, primitives -> 48-B float
// records), tile rendering, batched ray queries, counters.
//
// Replaces CUDAPathTracer (cuda_src/setup.h:90-148, setup.cu:92-843): instead of
// one cudaMalloc+cudaMemcpy per BVH node (setup.cu:429-476), constant-memory
// tables capped at 20 entries (kernel.cu:3-20) and exit() on error, the scene is
// flattened on the host into four contiguous arrays, uploaded once, and every
// failure is returned as a PT_E_* code with a message in pt_last_error().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ptgpu.h"
#include "../../include/ptgpu_scene.h"
#include "pt_device.h"
#include "pt_error.h"

namespace {

int fail(int code, const std::string& msg) { return pt_fail(code, msg); }

#define HIPCHK(expr)                                                                            \
  do {                                                                                          \
    hipError_t _e = (expr);                                                                     \
    if (_e != hipSuccess) return fail(PT_E_HIP, std::string(#expr ": ") + hipGetErrorString(_e)); \
  } while (0)

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  hipError_t reserve(size_t count) {
    if (count <= n && p) return hipSuccess;
    if (p) {  // renders in flight on other streams may still read the old array
      (void)hipDeviceSynchronize();
      (void)hipFree(p);
    }
    p = nullptr;
    n = 0;
    hipError_t e = hipMalloc(&p, std::max<size_t>(count, 1) * sizeof(T));
    if (e == hipSuccess) n = std::max<size_t>(count, 1);
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  void adopt(T* q, size_t count) {  // take ownership of a hipMalloc'd array
    release();
    p = q;
    n = count;
  }
};

float round_down(double x) {
  float f = (float)x;
  if ((double)f > x) f = std::nextafter(f, -INFINITY);
  return f;
}
float round_up(double x) {
  float f = (float)x;
  if ((double)f < x) f = std::nextafter(f, INFINITY);
  return f;
}

// EnvironmentLight's constructor tables (environment_light.cpp:6-48) in its own
// float arithmetic and summation order, so the GPU's inverse-CDF sampling
// picks the same texel as the reference for the same (r1, r2):
//   pThetaPhi[y][x] = illum * sin(theta_y) / C, pTheta = running row sums,
//   pPhiGivenTheta = running sums of pThetaPhi / pTheta[y] within the row.
struct EnvTables {
  std::vector<float4> tex;
  std::vector<float> p_theta, p_phi, p_theta_phi;
  std::vector<int> g_theta, g_phi;  // guide tables (PT_ENV_GUIDE buckets)
  std::vector<EnvRec> r_theta, r_phi;  // their bucket records
};

// g[k] = lower_bound(a, k/G * a[n-1]), k = 0..G
static void build_guide(const float* a, int n, int* g) {
  const float total = a[n - 1];
  for (int k = 0; k <= PT_ENV_GUIDE; ++k) {
    const float v = (float)((double)k / PT_ENV_GUIDE) * total;
    g[k] = (int)(std::lower_bound(a, a + n, v) - a);
    if (g[k] > n - 1) g[k] = n - 1;
  }
}
// The bucket records of a (n entries) from its guide table g (EnvRec).
static void build_records(const float* a, const int* g, EnvRec* r) {
  for (int k = 0; k < PT_ENV_GUIDE; ++k) {
    EnvRec& e = r[k];
    e.lo = g[std::max(k - 1, 0)];
    e.hi = g[std::min(k + 2, PT_ENV_GUIDE)];
    e.wm = e.lo > 0 ? a[e.lo - 1] : 0.0f;
    e.w0 = a[std::min(e.lo, e.hi)];
    e.w1 = a[std::min(e.lo + 1, e.hi)];
    e.w2 = a[std::min(e.lo + 2, e.hi)];
    e.w3 = a[std::min(e.lo + 3, e.hi)];
    e.w4 = a[e.hi];
  }
}
#pragma clang fp contract(off)
void build_env_tables(const float* rgb, int w, int h, EnvTables& t) {
  const double kPi = 3.14159265358979323;  // CMU462 PI
  t.tex.resize((size_t)w * h);
  t.p_theta.assign((size_t)h, 0.f);
  t.p_phi.assign((size_t)w * h, 0.f);
  t.p_theta_phi.assign((size_t)w * h, 0.f);
  for (size_t i = 0; i < (size_t)w * h; ++i) t.tex[i] = make_float4(rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2], 0.f);
  float C = 0;
  for (int y = 0; y < h; y++) {
    float theta = (y + 0.5) / h * kPi;
    float sin_theta = std::sin((double)theta);
    for (int x = 0; x < w; x++) {
      const float* p = rgb + 3 * ((size_t)x + (size_t)w * y);
      float illum = 0.2126f * p[0] + 0.7152f * p[1] + 0.0722f * p[2];  // Spectrum::illum
      t.p_theta_phi[(size_t)y * w + x] = illum * sin_theta;
      C += t.p_theta_phi[(size_t)y * w + x];
    }
  }
  for (int y = 0; y < h; y++) {
    for (int x = 0; x < w; x++) {
      t.p_theta_phi[(size_t)y * w + x] /= C;
      t.p_theta[y] += t.p_theta_phi[(size_t)y * w + x];
    }
    if (t.p_theta[y] != 0)
      for (int x = 0; x < w; x++) t.p_phi[(size_t)y * w + x] = t.p_theta_phi[(size_t)y * w + x] / t.p_theta[y];
  }
  for (int y = 0; y < h; y++) {
    if (y > 0) t.p_theta[y] += t.p_theta[y - 1];
    for (int x = 1; x < w; x++) t.p_phi[(size_t)y * w + x] += t.p_phi[(size_t)y * w + x - 1];
  }
  t.g_theta.resize(PT_ENV_GUIDE + 1);
  build_guide(t.p_theta.data(), h, t.g_theta.data());
  t.g_phi.resize((size_t)h * (PT_ENV_GUIDE + 1));
  for (int y = 0; y < h; y++) build_guide(&t.p_phi[(size_t)y * w], w, &t.g_phi[(size_t)y * (PT_ENV_GUIDE + 1)]);
  t.r_theta.resize(PT_ENV_GUIDE);
  build_records(t.p_theta.data(), t.g_theta.data(), t.r_theta.data());
  t.r_phi.resize((size_t)h * PT_ENV_GUIDE);
  for (int y = 0; y < h; y++)
    build_records(&t.p_phi[(size_t)y * w], &t.g_phi[(size_t)y * (PT_ENV_GUIDE + 1)], &t.r_phi[(size_t)y * PT_ENV_GUIDE]);
}

// Render-slot streams: plain non-blocking streams at normal priority.  HIP
// keeps one pool of GPU_MAX_HW_QUEUES (= 4) hardware queues per stream
// priority and gives a new stream the least-used queue of its pool; kernel
// traces and A/Bs of the C3 split's shares (profiles/r6/ab_stream_queues.txt)
// put render slots at high priority, on CU-masked queues of their own, or
// the caller's stream at high priority: every arm that keeps more than four
// hardware queues busy -- counting torch's collective stream on a rank of an
// N-GPU run -- was slower (N = 8 share 0.22 -> 0.29-0.38 ms per frame).
static hipError_t make_render_stream(hipStream_t* s) { return hipStreamCreateWithFlags(s, hipStreamNonBlocking); }

#pragma clang fp contract(on)

}  // namespace

struct pt_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  // launch timing: a ring of (render start, render end, resolve end) event
  // triples so device renders need not synchronise (pt_get_launch_times)
  static constexpr int kRing = 256;
  hipEvent_t ev[kRing][3] = {};
  int64_t n_launches = 0;   // launches recorded so far (ring slot = index % kRing)
  bool census_valid = false;  // the last launch was a PT_CENSUS plain launch (its trace area holds start/end/CU)
  bool times_pending = false;  // c->last's times belong to a launch not yet synchronised
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;  // the current launch's triple
  DevBuf<DNode> nodes;    // the render tree (BVH4)
  DevBuf<DNode2> nodes2;  // binary tree for PT_FLAG_REF_COUNTS
  DevBuf<int> prim_map;   // own BVH order (SAH or GPU-built) -> uploaded primitive index (else empty)
  // primitives in the caller's (reference BVH) order, for the reference-count
  // launch over nodes2 when the render tree is our own (else empty)
  DevBuf<DPrim> prims_ref;
  DevBuf<float> norms_ref;
  DevBuf<float4> env_tex;          // environment map RGB (w*h, .w unused)
  DevBuf<float> env_ptheta, env_pphi, env_pdf;  // EnvironmentLight tables
  DevBuf<EnvRec> env_rtheta, env_rphi;            // their guide tables' bucket records
  int env_w = 0, env_h = 0;
  DevBuf<DPrim> prims;
  DevBuf<float> norms;
  DevBuf<DBsdf> bsdfs;
  DevBuf<DLight> lights;
  // Render pipeline: launches alternate between kSlots slots, each with its
  // own render stream and per-launch device state (tile and block lists,
  // work-queue heads, sample-group sums, stack spill area).  A render waits
  // only until the resolve of the previous launch of ITS slot has consumed
  // the slot's group sums (ev_free), so consecutive device renders overlap:
  // the next frame's waves fill the CUs the previous frame's drain leaves
  // idle.  Each resolve runs on the caller's stream after its own render, so
  // the caller's stream order is kept for everything it can observe.
  // Small launches (a strong split's share of a frame: few work slots per
  // resident lane) rotate over all kSlots slots, so up to four frames are in
  // flight; larger ones over the first two (three slots measured C3 -6%, four
  // -10%: profiles/r6/ab_render_slots.txt).  See launch(): small launches.
  static constexpr int kSlots = 4;
  static constexpr int kSlotsLarge = 2;
  uint64_t slot_rr = 0;      // launches issued on the pipeline (slot rotation)
  bool small_last = false;   // the previous launch was small: rotate over every slot
  hipStream_t rstream[kSlots] = {};
  hipEvent_t ev_free[kSlots] = {};
  DevBuf<int4> tiles[kSlots];
  std::vector<int4> tiles_host[kSlots];  // what `tiles` holds
  DevBuf<int4> blocks[kSlots];           // footprint-clipped 8x8 pixel blocks of the tiles
  std::vector<int4> blocks_host[kSlots];
  DevBuf<int> tblock0[kSlots];           // first block of each tile (+ the end), for the resolve
  std::vector<int> tblock0_host[kSlots];
  DevBuf<int> tout[kSlots];              // caller's index of each launched tile (a Z-ordered packed launch)
  std::vector<int> tout_host[kSlots];
  DevBuf<float> partial[kSlots];   // per-slot sample-group sums
  DevBuf<int> spill[kSlots];       // traversal stack entries beyond PT_STACK
  DevBuf<uint32_t> counter[kSlots];
  // the slot's queue heads are known to be zero: the last resolve of the slot
  // reset them (PT_RESOLVE_RESETS), so the next launch needs no memset
  bool counter_clean[kSlots] = {};
  int64_t culled_px = 0;         // pixels of the last launch outside the footprint
  DevBuf<float> frame;  // device framebuffer for host-output renders
  // Asynchronous one-tile seam (pt_tile_submit / pt_tile_finish): submitted
  // tiles wait in `tq` until a batch of `tile_batch` is full, then render as
  // ONE launch into `frame`; the rows the batch spans are copied to the
  // batch's own pinned stage and an event is recorded behind the copy.  A
  // completion thread (`tworker`) waits on that event and completes the
  // batch -- copies its tiles into the caller's sampleBuffer and toColors them
  // into its frameBuffer -- OFF the stream, so the next batch's render never
  // waits for host work (a stream host function would serialise them).
  struct TileJob {
    int4 t;
    float* hdr;
    uint32_t* rgba;
  };
  struct TileBatch {
    std::vector<TileJob> jobs;
    float* stage = nullptr;  // pinned: rows y0 .. y0 + rows - 1 of the frame
    size_t cap = 0;          // floats the stage holds
    int y0 = 0, W = 0, H = 0;
    hipEvent_t ev = nullptr;
  };
  std::vector<TileJob> tq;
  int tile_batch = 256;  // tiles per launch (PT_TILE_BATCH): 256 beat 16-128 and 1024 (profiles/r3/seam_native_batch_sweep.txt)
  int fault_tile_launch = 0, n_tile_launches = 0;  // PT_FAULT_TILE_LAUNCH (tests)
  std::mutex tmu;
  std::condition_variable tcv;
  std::deque<TileBatch*> tpending;  // rendered batches awaiting completion, in launch order
  std::vector<TileBatch*> tfree;    // completed batches: stages and events for reuse
  int tinflight = 0;                // batches launched and not yet completed
  int terr = PT_OK;                 // first completion error (reported by pt_tile_finish)
  std::string terrmsg;
  bool tstop = false;
  std::thread tworker;
  DevBuf<int> q_spill;  // ray-query stack spill
  DevBuf<unsigned long long> stats;
  DevBuf<float> q_f;    // ray-query scratch
  DevBuf<int32_t> q_i;
  int n_lights = 0, n_bsdfs = 0;
  int bvh_stack = 0;  // worst-case traversal stack entries of the uploaded BVH
  size_t n_render_nodes = 0;
  int64_t n_prims = 0;
  bool tri_only = false;  // every primitive a triangle
  float root_lo[3] = {0, 0, 0}, root_hi[3] = {0, 0, 0};
  double root_lo_d[3] = {0, 0, 0}, root_hi_d[3] = {0, 0, 0};
  bool have_scene = false, have_cam = false, have_params = false;
  pt_camera cam{};
  pt_params params{};
  pt_stats last{};
  int grid_plain = 0, grid_stats = 0;
  int bpc_plain = 0, bpc_stats = 0, n_cu = 0;
  int bpc_variant[4] = {0, 0, 0, 0};  // plain builds: [env * 2 + gtab] (the common one is bpc_plain)
};

extern "C" {


int pt_create(int device, pt_ctx** out) {
  if (!out) return fail(PT_E_INVALID, "pt_create: out is NULL");
  *out = nullptr;
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(PT_E_INVALID, "pt_create: no such HIP device");
  HIPCHK(hipSetDevice(device));
  pt_ctx* c = new pt_ctx();
  c->device = device;
  HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  for (int k = 0; k < pt_ctx::kSlots; ++k) {
    // (slots past the first two get their stream when a small launch first
    // uses them: HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues, 4 by
    // default, and two more streams per context put the render streams of
    // large frames on shared queues -- C3 pipelined -12%)
    if (k < pt_ctx::kSlotsLarge) {
      HIPCHK(make_render_stream(&c->rstream[k]));
      HIPCHK(hipEventCreateWithFlags(&c->ev_free[k], hipEventDisableTiming));
      HIPCHK(hipEventRecord(c->ev_free[k], c->stream));
    }
    HIPCHK(c->counter[k].reserve(PT_QUEUE_WORDS * PT_QUEUE_HEADS));  // work-queue heads, one 128-B line each
  }
  for (auto& tri : c->ev)
    for (auto& e : tri) HIPCHK(hipEventCreate(&e));
  HIPCHK(c->stats.reserve(PT_STATS_SLOTS));
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, device));
  // Persistent grid: as many one-wave workgroups as can be resident.  The
  // work queue needs no co-residency (no grid barrier), so a wrong occupancy
  // answer only costs speed; never size below 8 waves per CU.
  c->n_cu = prop.multiProcessorCount;
  HIPCHK(ptk_render_occupancy(&c->bpc_plain, false, false, false));
  HIPCHK(ptk_render_occupancy(&c->bpc_stats, true, false, false));
  for (int v = 0; v < 4; ++v) HIPCHK(ptk_render_occupancy(&c->bpc_variant[v], false, (v & 2) != 0, (v & 1) != 0));
  c->grid_plain = std::max(8, c->bpc_plain) * c->n_cu;
  c->grid_stats = std::max(8, c->bpc_stats) * c->n_cu;
  if (const char* tb = std::getenv("PT_TILE_BATCH")) {  // tuning knob: tiles per asynchronous launch
    int v = std::atoi(tb);
    if (v >= 1) c->tile_batch = v;
  }
  if (const char* f = std::getenv("PT_FAULT_TILE_LAUNCH")) c->fault_tile_launch = std::atoi(f);
  // counters + one trace record per wave of the largest stats grid
  HIPCHK(c->stats.reserve(PT_STATS_SLOTS + (size_t)PT_WAVE_TRACE * std::max(c->grid_stats, 64 * c->n_cu)));
  *out = c;
  return PT_OK;
}

static void tile_worker_stop(pt_ctx* c);

int pt_destroy(pt_ctx* c) {
  if (!c) return PT_OK;
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();  // no render of this context may still be running
  c->nodes.release();
  c->nodes2.release();
  c->prim_map.release();
  c->env_tex.release();
  c->env_ptheta.release();
  c->env_pphi.release();
  c->env_pdf.release();
  c->env_rtheta.release();
  c->env_rphi.release();
  c->prims.release();
  c->norms.release();
  c->bsdfs.release();
  c->lights.release();
  for (int k = 0; k < pt_ctx::kSlots; ++k) {
    c->tiles[k].release();
    c->blocks[k].release();
    c->tblock0[k].release();
    c->tout[k].release();
    c->spill[k].release();
    c->partial[k].release();
    c->counter[k].release();
    if (c->ev_free[k]) (void)hipEventDestroy(c->ev_free[k]);
    if (c->rstream[k]) (void)hipStreamDestroy(c->rstream[k]);
  }
  tile_worker_stop(c);
  c->q_spill.release();
  c->frame.release();
  c->stats.release();
  c->q_f.release();
  c->q_i.release();
  for (auto& tri : c->ev)
    for (auto& e : tri)
      if (e) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return PT_OK;
}

// Reference BVH (pt_scene.nodes) -> BVH4 nodes (dn), binary nodes (d2) and
// the worst-case traversal stack.
static int build_host_bvh(const pt_scene* s, std::vector<DNode>& dn, std::vector<DNode2>& d2, int& max_stack) {
  // ---- BVH: internal nodes only, pre-order, child boxes rounded outward;
  // leaves become cursors in their parent's child references.  Leaves of more
  // than 8 primitives are split into small subtrees over primitive boxes.
  const pt_bvh_node* N = s->nodes;
  const int64_t nn = s->n_nodes;
  auto is_leaf = [&](int64_t i) { return N[i].left < 0 && N[i].right < 0; };
  for (int64_t i = 0; i < nn; ++i) {
    if ((N[i].left < 0) != (N[i].right < 0)) return fail(PT_E_INVALID, "pt_upload_scene: half-empty BVH node");
    if (N[i].left >= nn || N[i].right >= nn) return fail(PT_E_INVALID, "pt_upload_scene: BVH child out of range");
    if (is_leaf(i) && (N[i].start < 0 || N[i].range <= 0 || N[i].start + N[i].range > s->n_prims))
      return fail(PT_E_INVALID, "pt_upload_scene: bad leaf range");
  }
  if (s->n_prims >= ((int64_t)1 << 27)) return fail(PT_E_INVALID, "pt_upload_scene: too many primitives for leaf cursors");
  auto prim_box = [&](int64_t first, int64_t count, double lo[3], double hi[3]) {
    for (int k = 0; k < 3; ++k) {
      lo[k] = INFINITY;
      hi[k] = -INFINITY;
    }
    for (int64_t i = first; i < first + count; ++i) {
      const double* g = s->prim_geom + 9 * i;
      for (int k = 0; k < 3; ++k) {
        if (s->prim_type[i] == PT_PRIM_TRIANGLE) {
          lo[k] = std::min({lo[k], g[k], g[3 + k], g[6 + k]});
          hi[k] = std::max({hi[k], g[k], g[3 + k], g[6 + k]});
        } else {
          lo[k] = std::min(lo[k], g[k] - std::fabs(g[3]));
          hi[k] = std::max(hi[k], g[k] + std::fabs(g[3]));
        }
      }
    }
  };
  // a subtree to emit: a reference node, or a primitive range (split leaf)
  struct Sub {
    int64_t ref;          // >= 0: reference node; -1: primitive range
    int64_t first, count;
    double lo[3], hi[3];
  };
  auto sub_of_node = [&](int64_t r) {
    Sub u{r, N[r].start, N[r].range, {}, {}};
    for (int k = 0; k < 3; ++k) {
      u.lo[k] = N[r].bb_min[k];
      u.hi[k] = N[r].bb_max[k];
    }
    return u;
  };
  auto sub_of_range = [&](int64_t first, int64_t count) {
    Sub u{-1, first, count, {}, {}};
    prim_box(first, count, u.lo, u.hi);
    return u;
  };
  auto sub_is_leaf = [&](const Sub& u) { return u.ref >= 0 ? is_leaf(u.ref) && u.count <= 8 : u.count <= 8; };
  auto sub_children = [&](const Sub& u, Sub ch[2]) {
    if (u.ref >= 0 && !is_leaf(u.ref)) {
      ch[0] = sub_of_node(N[u.ref].left);
      ch[1] = sub_of_node(N[u.ref].right);
    } else {  // oversized leaf: halve the primitive range
      int64_t h = u.count / 2;
      ch[0] = sub_of_range(u.first, h);
      ch[1] = sub_of_range(u.first + h, u.count - h);
    }
  };
  // (1) binary tree over the reference topology: child boxes rounded outward
  // to fp32, child references are node indices or leaf cursors
  struct B2 {
    float lo[2][3], hi[2][3];
    int ref[2];
  };
  auto set_box = [&](B2& d, int side, const Sub& u) {
    for (int k = 0; k < 3; ++k) {
      d.lo[side][k] = round_down(u.lo[k]);
      d.hi[side][k] = round_up(u.hi[k]);
    }
  };
  auto cursor = [](int64_t first, int64_t count) { return (int)~((first << 3) | (count - 1)); };
  std::vector<B2> b2;
  Sub root = sub_of_node(0);
  if (sub_is_leaf(root)) {  // one leaf: a root whose second child box is empty
    B2 d{};
    set_box(d, 0, root);
    for (int k = 0; k < 3; ++k) d.lo[1][k] = d.hi[1][k] = INFINITY;
    d.ref[0] = cursor(root.first, root.count);
    // the empty child is a leaf cursor (never entered: its box is at +inf),
    // never a node reference -- node 0 as its own child would be opened and
    // pushed forever by the collapse below
    d.ref[1] = cursor(0, 1);
    b2.push_back(d);
  } else {
    // explicit DFS: (subtree, parent node, side)
    struct Item { Sub u; int64_t parent; int side; };
    std::vector<Item> st = {{root, -1, 0}};
    while (!st.empty()) {
      Item it = st.back();
      st.pop_back();
      int64_t me = (int64_t)b2.size();
      b2.push_back(B2{});
      if (it.parent >= 0) b2[it.parent].ref[it.side] = (int)me;
      Sub ch[2];
      sub_children(it.u, ch);
      for (int side = 0; side < 2; ++side) {
        set_box(b2[me], side, ch[side]);
        if (sub_is_leaf(ch[side])) b2[me].ref[side] = cursor(ch[side].first, ch[side].count);
      }
      for (int side = 1; side >= 0; --side)
        if (!sub_is_leaf(ch[side])) st.push_back({ch[side], me, side});
    }
  }
  if ((int64_t)b2.size() >= ((int64_t)1 << 31)) return fail(PT_E_INVALID, "pt_upload_scene: too many BVH nodes");

  // (2) collapse to 4-wide nodes: repeatedly open the internal child of the
  // largest surface area (the usual BVH2 -> BVH4 collapse).  Pre-order, so
  // a node's first child follows it in memory.
  struct Child {
    float lo[3], hi[3];
    int ref;
  };
  auto area = [](const Child& c) {
    float dx = c.hi[0] - c.lo[0], dy = c.hi[1] - c.lo[1], dz = c.hi[2] - c.lo[2];
    return dx * dy + dy * dz + dz * dx;
  };
  auto kids = [&](int n, Child out[2]) {
    for (int s2 = 0; s2 < 2; ++s2) {
      for (int k = 0; k < 3; ++k) {
        out[s2].lo[k] = b2[(size_t)n].lo[s2][k];
        out[s2].hi[k] = b2[(size_t)n].hi[s2][k];
      }
      out[s2].ref = b2[(size_t)n].ref[s2];
    }
  };
  // primitives under each binary node (b2 is pre-order: children follow parents)
  std::vector<double> under(b2.size(), 0.0);
  for (size_t i = b2.size(); i-- > 0;)
    for (int s2 = 0; s2 < 2; ++s2) {
      const int r = b2[i].ref[s2];
      under[i] += r >= 0 ? under[(size_t)r] : (double)(((~r) & 7) + 1);
    }
  // The collapse: PT_COLLAPSE=dp (default for the host trees: the SAH-optimal
  // choice of the binary nodes kept as BVH4 nodes, the DP of lbvh.hip's k_dp;
  // C3 over the host SAH tree 46.2 -> 51.0 G samples/s, +10%:
  // profiles/r5/ab_collapse_dp.txt), or greedy -- open the internal child with
  // the largest surface area (area), the most primitives (count) or area x
  // primitives (sah) until four.
  const char* cm = std::getenv("PT_COLLAPSE");
  const int crit = !cm || std::strcmp(cm, "dp") == 0 ? 3
                   : std::strcmp(cm, "count") == 0   ? 1
                   : std::strcmp(cm, "sah") == 0     ? 2
                                                     : 0;
  // DP tables (crit 3): dpc[4n + i-1] = least expected steps of binary node
  // n's subtree in <= i slots (a node or a two-primitive leaf step costs one,
  // weighted by area); dpk = slots for its left child, -1 = as with i - 1
  std::vector<double> dpc;
  std::vector<int8_t> dpk;
  if (crit == 3) {
    dpc.assign(b2.size() * 4, 0.0);
    dpk.assign(b2.size() * 4, 0);
    auto box_area = [](const float lo[3], const float hi[3]) {
      const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
      return dx * dy + dy * dz + dz * dx;
    };
    for (size_t n = b2.size(); n-- > 0;) {  // (pre-order: children after parents)
      double a[2][5];
      for (int s2 = 0; s2 < 2; ++s2) {
        const int r = b2[n].ref[s2];
        for (int i = 1; i <= 4; ++i)
          a[s2][i] = r >= 0 ? dpc[(size_t)r * 4 + (i - 1)]
                            : box_area(b2[n].lo[s2], b2[n].hi[s2]) * (double)((((~r) & 7) + 2) / 2);
      }
      double dist[5];
      int8_t arg[5];
      for (int j = 2; j <= 4; ++j) {
        dist[j] = INFINITY;
        arg[j] = 1;
        for (int k = 1; k < j; ++k)
          if (a[0][k] + a[1][j - k] < dist[j]) {
            dist[j] = a[0][k] + a[1][j - k];
            arg[j] = (int8_t)k;
          }
      }
      float ulo[3], uhi[3];
      for (int k = 0; k < 3; ++k) {
        ulo[k] = std::min(b2[n].lo[0][k], b2[n].lo[1][k]);
        uhi[k] = std::max(b2[n].hi[0][k], b2[n].hi[1][k]);
      }
      double prev = box_area(ulo, uhi) + dist[4];
      dpc[n * 4] = prev;
      dpk[n * 4] = arg[4];
      for (int i = 2; i <= 4; ++i) {
        const bool open = dist[i] < prev;
        prev = open ? dist[i] : prev;
        dpc[n * 4 + (i - 1)] = prev;
        dpk[n * 4 + (i - 1)] = open ? arg[i] : (int8_t)-1;
      }
    }
  }
  // the DP's children of binary node b kept whole: its two children over four
  // slots, each opened as its table says, in left-to-right order
  auto dp_kids = [&](int b, Child out[4]) -> int {
    int sp = 0, n = 0, sb[8], ss[8], si[8];
    const int k4 = dpk[(size_t)b * 4];
    sb[sp] = b; ss[sp] = 1; si[sp++] = 4 - k4;
    sb[sp] = b; ss[sp] = 0; si[sp++] = k4;
    while (sp > 0) {
      --sp;
      const int pb = sb[sp], side = ss[sp];
      int i = si[sp];
      const int r = b2[(size_t)pb].ref[side];
      if (r >= 0) {
        while (i > 1 && dpk[(size_t)r * 4 + (i - 1)] == -1) --i;
        if (i > 1) {
          const int k = dpk[(size_t)r * 4 + (i - 1)];
          sb[sp] = r; ss[sp] = 1; si[sp++] = i - k;
          sb[sp] = r; ss[sp] = 0; si[sp++] = k;
          continue;
        }
      }
      Child c;
      for (int k = 0; k < 3; ++k) {
        c.lo[k] = b2[(size_t)pb].lo[side][k];
        c.hi[k] = b2[(size_t)pb].hi[side][k];
      }
      c.ref = r;
      out[n++] = c;
    }
    return n;
  };
  auto weight = [&](const Child& c) {
    const double n = c.ref >= 0 ? under[(size_t)c.ref] : 0.0;
    return crit == 0 ? (double)area(c) : crit == 1 ? n : (double)area(c) * n;
  };
  max_stack = 0;
  {
    struct Item4 { int b2node; int64_t parent; int slot; int stack; };
    std::vector<Item4> st = {{0, -1, 0, 0}};
    while (!st.empty()) {
      Item4 it = st.back();
      st.pop_back();
      Child ch[4];
      int n = 2;
      if (crit == 3) {
        n = dp_kids(it.b2node, ch);
      } else {
      kids(it.b2node, ch);
      while (n < 4) {
        int best = -1;
        double ba = -1.0;
        for (int k = 0; k < n; ++k)
          if (ch[k].ref >= 0 && weight(ch[k]) > ba) {
            ba = weight(ch[k]);
            best = k;
          }
        if (best < 0) break;
        Child two[2];
        kids(ch[best].ref, two);
        ch[best] = two[0];
        ch[n++] = two[1];
      }
      }
      int64_t me = (int64_t)dn.size();
      dn.push_back(DNode{});
      if (it.parent >= 0) (&dn[(size_t)it.parent].ref.x)[it.slot] = (int)me;
      DNode& d = dn[(size_t)me];
      float* lox = &d.lox.x; float* hix = &d.hix.x; float* loy = &d.loy.x;
      float* hiy = &d.hiy.x; float* loz = &d.loz.x; float* hiz = &d.hiz.x;
      int* ref = &d.ref.x;
      for (int k = 0; k < 4; ++k) {
        if (k < n) {
          lox[k] = ch[k].lo[0]; hix[k] = ch[k].hi[0];
          loy[k] = ch[k].lo[1]; hiy[k] = ch[k].hi[1];
          loz[k] = ch[k].lo[2]; hiz[k] = ch[k].hi[2];
          ref[k] = ch[k].ref;
        } else {  // empty slot: the box at +inf, which no ray enters (an inverted
                  // box would not do: the slab test orders each pair of planes)
          lox[k] = loy[k] = loz[k] = hix[k] = hiy[k] = hiz[k] = INFINITY;
          ref[k] = 0;
        }
      }
      // a visit pushes at most n-1 siblings before descending
      const int below = it.stack + (n - 1);
      max_stack = std::max(max_stack, below);
      for (int k = n - 1; k >= 0; --k)
        if (ch[k].ref >= 0) st.push_back({ch[k].ref, me, k, below});
    }
  }
  if (std::getenv("PT_BVH_REPORT")) {
    // expected steps per random ray (surface-area heuristic over the BVH4):
    // node steps = sum of node areas / root area; leaf steps = sum over
    // leaves of area * ceil(count / 2) / root area
    auto a3 = [](float lx, float hx, float ly, float hy, float lz, float hz) {
      const double dx = hx - lx, dy = hy - ly, dz = hz - lz;
      return dx * dy + dy * dz + dz * dx;
    };
    double root = 0, nodes = 0, leaves = 0;
    for (size_t i = 0; i < dn.size(); ++i) {
      const DNode& d = dn[i];
      for (int k = 0; k < 4; ++k) {
        if (std::isinf((&d.lox.x)[k])) continue;
        const double a = a3((&d.lox.x)[k], (&d.hix.x)[k], (&d.loy.x)[k], (&d.hiy.x)[k], (&d.loz.x)[k], (&d.hiz.x)[k]);
        root += i == 0 ? a : 0.0;
        const int r = (&d.ref.x)[k];
        if (r >= 0) nodes += a;
        else leaves += a * (double)((((~r) & 7) + 2) / 2);
      }
    }
    std::fprintf(stderr, "[pt] BVH4: %zu nodes, stack %d, SAH node steps %.3f leaf steps %.3f (per root-box ray)\n",
                 dn.size(), max_stack, (nodes + root) / root, leaves / root);
  }
  // Traversal termination rests on this: node references only point forward
  // (pre-order), so a ray can never re-enter a node it has left.
  for (size_t i = 0; i < dn.size(); ++i)
    for (int k = 0; k < 4; ++k) {
      int r = (&dn[i].ref.x)[k];
      bool empty = std::isinf((&dn[i].lox.x)[k]);
      if (!empty && r >= 0 && (r <= (int)i || r >= (int)dn.size()))
        return fail(PT_E_INVALID, "pt_upload_scene: BVH4 child reference is not forward");
    }
  if (max_stack > PT_STACK_MAX)
    return fail(PT_E_INVALID, "pt_upload_scene: BVH needs a deeper traversal stack (" + std::to_string(max_stack) +
                                  " > " + std::to_string(PT_STACK_MAX) + ")");

  d2.resize(b2.size());
  for (size_t i = 0; i < b2.size(); ++i) {
    const B2& q = b2[i];
    d2[i].a = make_float4(q.lo[0][0], q.hi[0][0], q.lo[0][1], q.hi[0][1]);
    d2[i].b = make_float4(q.lo[1][0], q.hi[1][0], q.lo[1][1], q.hi[1][1]);
    d2[i].c = make_float4(q.lo[0][2], q.hi[0][2], q.lo[1][2], q.hi[1][2]);
    d2[i].e = make_int4(q.ref[0], q.ref[1], 0, 0);
  }
  return PT_OK;
}

// GPU linear-BVH build over the primitives already in c->prims / c->norms
// (CUDAPathTracer::buildBVH, cuda_src/setup.cu:478-686; kernels in lbvh.hip).
static int build_gpu_bvh(pt_ctx* c, const pt_scene* s) {
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int64_t i = 0; i < s->n_prims; ++i) {  // sceneBox.expand(prim->get_bbox()) (setup.cu:482-487)
    const double* g = s->prim_geom + 9 * i;
    for (int k = 0; k < 3; ++k) {
      if (s->prim_type[i] == PT_PRIM_TRIANGLE) {
        lo[k] = std::min({lo[k], g[k], g[3 + k], g[6 + k]});
        hi[k] = std::max({hi[k], g[k], g[3 + k], g[6 + k]});
      } else {
        lo[k] = std::min(lo[k], g[k] - std::fabs(g[3]));
        hi[k] = std::max(hi[k], g[k] + std::fabs(g[3]));
      }
    }
  }
  LbvhIn in{};
  in.n = (int)s->n_prims;
  in.prims = c->prims.p;
  in.norms = c->norms.p;
  for (int k = 0; k < 3; ++k) {
    in.scene_min[k] = round_down(lo[k]);
    in.scene_extent[k] = (float)(hi[k] - lo[k]);
  }
  LbvhOut out{};
  HIPCHK(ptk_build_lbvh(&in, &out, c->stream));
  c->prims.adopt(out.prims, (size_t)in.n);
  c->norms.adopt(out.norms, (size_t)in.n * 9);
  c->prim_map.adopt(out.prim_map, (size_t)in.n);
  c->nodes.adopt(out.nodes4, (size_t)out.n4);
  c->nodes2.adopt(out.nodes2, (size_t)std::max(1, out.n2));
  c->n_render_nodes = (size_t)out.n4;
  if (out.max_stack > PT_STACK_MAX)
    return fail(PT_E_INVALID, "pt_upload_scene_lbvh: BVH needs a deeper traversal stack (" +
                                  std::to_string(out.max_stack) + " > " + std::to_string(PT_STACK_MAX) + ")");
  c->bvh_stack = out.max_stack;
  for (int k = 0; k < 3; ++k) {
    c->root_lo[k] = out.root_lo[k];
    c->root_hi[k] = out.root_hi[k];
    c->root_lo_d[k] = out.root_lo[k];
    c->root_hi_d[k] = out.root_hi[k];
  }
  return PT_OK;
}

static int tile_launch(pt_ctx* c);

static int upload_impl(pt_ctx* c, const pt_scene* s, bool gpu_bvh) {
  if (!c || !s) return fail(PT_E_INVALID, "pt_upload_scene: NULL argument");
  if (int rc = tile_launch(c)) return rc;  // queued tiles render with the state they were submitted under
  if (s->n_prims <= 0 || !s->prim_type || !s->prim_bsdf || !s->prim_geom || !s->prim_norm ||
      (!gpu_bvh && (s->n_nodes <= 0 || !s->nodes)))
    return fail(PT_E_INVALID, "pt_upload_scene: empty scene");
  if (s->n_bsdfs <= 0 || !s->bsdfs) return fail(PT_E_INVALID, "pt_upload_scene: no BSDFs");
  if (s->n_lights < 0 || (s->n_lights > 0 && !s->lights)) return fail(PT_E_INVALID, "pt_upload_scene: bad lights");
  if (s->n_lights > 65535) return fail(PT_E_INVALID, "pt_upload_scene: more than 65535 lights");
  if (s->n_prims > (int64_t)0x3fffffff) return fail(PT_E_INVALID, "pt_upload_scene: too many primitives");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipDeviceSynchronize());  // renders in flight read the scene being replaced

  // Own SAH tree (PT_BVH_BUILD=sah): the primitives are permuted into its
  // leaf order and uploaded that way; prim_map takes ray-query ids back.
  std::vector<pt_bvh_node> sah_nodes;
  std::vector<int64_t> perm;
  std::vector<int32_t> ptype, pbsdf;
  std::vector<double> pgeom, pnorm;
  pt_scene ps;
  const pt_scene* const s0 = s;  // the caller's scene (reference BVH order)
  int rc0 = 0;
  // The render tree: by default this library's GPU-built
  // tree (Karras LBVH + treelet restructuring, lbvh.hip) over the caller's
  // primitives; PT_BVH_BUILD=sah: the host binned-SAH tree; =ref: the
  // caller's own (reference) tree.  pt_upload_scene_lbvh always builds on
  // the GPU.  The reference-count launch walks the caller's tree in every case
  // but pt_upload_scene_lbvh's.
  const char* bb = std::getenv("PT_BVH_BUILD");
  const bool host_sah = bb && std::strcmp(bb, "sah") == 0;
  const bool ref_tree = bb && std::strcmp(bb, "ref") == 0;
  const bool gpu_tree = !gpu_bvh && !host_sah && !ref_tree;
  if (!gpu_bvh && host_sah) {
    sah_nodes.resize((size_t)std::max<int64_t>(1, 2 * s->n_prims - 1));
    perm.resize((size_t)s->n_prims);
    int64_t nn = 0;
    if (int rc = pt_host_build_render_tree(s, sah_nodes.data(), &nn, perm.data())) return rc;
    sah_nodes.resize((size_t)nn);
    const size_t np = (size_t)s->n_prims;
    ptype.resize(np);
    pbsdf.resize(np);
    pgeom.resize(np * 9);
    pnorm.resize(np * 9);
    for (size_t i = 0; i < np; ++i) {
      const size_t p = (size_t)perm[i];
      ptype[i] = s->prim_type[p];
      pbsdf[i] = s->prim_bsdf[p];
      std::memcpy(&pgeom[9 * i], s->prim_geom + 9 * p, 9 * sizeof(double));
      std::memcpy(&pnorm[9 * i], s->prim_norm + 9 * p, 9 * sizeof(double));
    }
    ps = *s;
    ps.prim_type = ptype.data();
    ps.prim_bsdf = pbsdf.data();
    ps.prim_geom = pgeom.data();
    ps.prim_norm = pnorm.data();
    ps.nodes = sah_nodes.data();
    ps.n_nodes = (int64_t)sah_nodes.size();
    s = &ps;
  }

  // ---- primitives (already in BVH order)
  std::vector<DPrim> prims, prims0;
  std::vector<float> norms, norms0;
  auto convert = [&](const pt_scene* s, std::vector<DPrim>& prims, std::vector<float>& norms) -> int {
  prims.resize((size_t)s->n_prims);
  norms.assign((size_t)s->n_prims * 9, 0.f);
  for (int64_t i = 0; i < s->n_prims; ++i) {
    const double* g = s->prim_geom + 9 * i;
    const double* n = s->prim_norm + 9 * i;
    int b = s->prim_bsdf[i];
    if (b < 0 || b >= s->n_bsdfs) return fail(PT_E_INVALID, "pt_upload_scene: primitive BSDF index out of range");
    DPrim& P = prims[(size_t)i];
    if (s->prim_type[i] == PT_PRIM_TRIANGLE) {
      int meta = (b << 1) | 1;
      float mf;
      std::memcpy(&mf, &meta, 4);
      P.v0 = make_float4((float)g[0], (float)g[1], (float)g[2], mf);
      P.e1 = make_float4((float)(g[3] - g[0]), (float)(g[4] - g[1]), (float)(g[5] - g[2]), 0.f);
      P.e2 = make_float4((float)(g[6] - g[0]), (float)(g[7] - g[1]), (float)(g[8] - g[2]), 0.f);
      for (int k = 0; k < 9; ++k) norms[9 * i + k] = (float)n[k];
    } else if (s->prim_type[i] == PT_PRIM_SPHERE) {
      int meta = (b << 1);
      float mf;
      std::memcpy(&mf, &meta, 4);
      P.v0 = make_float4((float)g[0], (float)g[1], (float)g[2], mf);
      P.e1 = make_float4((float)g[3], (float)(g[3] * g[3]), 0.f, 0.f);
      P.e2 = make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      return fail(PT_E_INVALID, "pt_upload_scene: unknown primitive type");
    }
  }
  return PT_OK;
  };
  if (int rc = convert(s, prims, norms)) return rc;
  if (s != s0 && (rc0 = convert(s0, prims0, norms0))) return rc0;

  std::vector<DBsdf> bs((size_t)s->n_bsdfs);
  for (int i = 0; i < s->n_bsdfs; ++i) {
    const pt_bsdf& B = s->bsdfs[i];
    if (B.type < 0 || B.type > 4) return fail(PT_E_INVALID, "pt_upload_scene: unknown BSDF type");
    DBsdf& d = bs[(size_t)i];
    d.type = B.type;
    for (int k = 0; k < 3; ++k) {
      d.a[k] = B.albedo[k];
      d.t[k] = B.transmittance[k];
      d.e[k] = B.emission[k];
    }
    d.ior = B.ior;
    d.pad = 0.f;
  }
  std::vector<DLight> ls((size_t)std::max(0, s->n_lights));
  int n_env = 0;
  for (int i = 0; i < s->n_lights; ++i) {
    const pt_light& L = s->lights[i];
    if (L.type < 0 || L.type > 4) return fail(PT_E_INVALID, "pt_upload_scene: unsupported light type");
    if (L.type == PT_LIGHT_ENVIRONMENT && ++n_env > 1)
      return fail(PT_E_INVALID, "pt_upload_scene: more than one environment light");
    DLight& d = ls[(size_t)i];
    std::memset(&d, 0, sizeof(d));
    d.type = L.type;
    for (int k = 0; k < 3; ++k) {
      d.rad[k] = L.radiance[k];
      d.pos[k] = (float)L.position[k];
      d.dir[k] = (float)L.direction[k];
      d.dimx[k] = (float)L.dim_x[k];
      d.dimy[k] = (float)L.dim_y[k];
    }
    d.area = L.area;
  }

  if (n_env && (!s->env_rgb || s->env_width <= 0 || s->env_height <= 0))
    return fail(PT_E_INVALID, "pt_upload_scene: environment light without a map (env_rgb/env_width/env_height)");
  if (!n_env && s->env_rgb) return fail(PT_E_INVALID, "pt_upload_scene: env_rgb given but no PT_LIGHT_ENVIRONMENT light");
  EnvTables env;
  if (n_env) build_env_tables(s->env_rgb, s->env_width, s->env_height, env);

  HIPCHK(c->prims.reserve(prims.size()));
  HIPCHK(c->norms.reserve(norms.size()));
  HIPCHK(c->bsdfs.reserve(bs.size()));
  HIPCHK(c->lights.reserve(std::max<size_t>(1, ls.size())));
  HIPCHK(hipMemcpy(c->prims.p, prims.data(), prims.size() * sizeof(DPrim), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(c->norms.p, norms.data(), norms.size() * sizeof(float), hipMemcpyHostToDevice));
  c->prim_map.release();
  c->prims_ref.release();
  c->norms_ref.release();
  if (!prims0.empty()) {
    HIPCHK(c->prims_ref.reserve(prims0.size()));
    HIPCHK(c->norms_ref.reserve(norms0.size()));
    HIPCHK(hipMemcpy(c->prims_ref.p, prims0.data(), prims0.size() * sizeof(DPrim), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->norms_ref.p, norms0.data(), norms0.size() * sizeof(float), hipMemcpyHostToDevice));
  }
  if (gpu_tree) {
    // the caller's tree: validated, kept as the binary nodes of the
    // reference-count launch over a caller-order copy of the primitives
    std::vector<DNode> dn0;
    std::vector<DNode2> d2;
    int ms0 = 0;
    if (int rc = build_host_bvh(s0, dn0, d2, ms0)) return rc;
    HIPCHK(c->prims_ref.reserve(prims.size()));
    HIPCHK(c->norms_ref.reserve(norms.size()));
    HIPCHK(hipMemcpy(c->prims_ref.p, prims.data(), prims.size() * sizeof(DPrim), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->norms_ref.p, norms.data(), norms.size() * sizeof(float), hipMemcpyHostToDevice));
    if (int rc = build_gpu_bvh(c, s0)) return rc;  // adopts prims/norms/prim_map/nodes in its own order
    HIPCHK(c->nodes2.reserve(d2.size()));
    HIPCHK(hipMemcpy(c->nodes2.p, d2.data(), d2.size() * sizeof(DNode2), hipMemcpyHostToDevice));
    c->bvh_stack = std::max(c->bvh_stack, ms0);
    if (c->bvh_stack > PT_STACK_MAX)
      return fail(PT_E_INVALID, "pt_upload_scene: BVH needs a deeper traversal stack (" +
                                    std::to_string(c->bvh_stack) + " > " + std::to_string(PT_STACK_MAX) + ")");
  } else if (!gpu_bvh) {
    std::vector<DNode> dn;
    std::vector<DNode2> d2;
    int max_stack = 0;
    int rc = build_host_bvh(s, dn, d2, max_stack);
    if (rc) return rc;
    if (s != s0) {  // the reference-count launch walks the caller's (reference) tree
      std::vector<DNode> dn0;
      int ms0 = 0;
      d2.clear();
      if ((rc = build_host_bvh(s0, dn0, d2, ms0))) return rc;
      max_stack = std::max(max_stack, ms0);
    }
    HIPCHK(c->nodes2.reserve(d2.size()));
    HIPCHK(hipMemcpy(c->nodes2.p, d2.data(), d2.size() * sizeof(DNode2), hipMemcpyHostToDevice));
    HIPCHK(c->nodes.reserve(dn.size()));
    HIPCHK(hipMemcpy(c->nodes.p, dn.data(), dn.size() * sizeof(DNode), hipMemcpyHostToDevice));
    if (!perm.empty()) {
      std::vector<int> pm(perm.begin(), perm.end());
      HIPCHK(c->prim_map.reserve(pm.size()));
      HIPCHK(hipMemcpy(c->prim_map.p, pm.data(), pm.size() * sizeof(int), hipMemcpyHostToDevice));
    }
    c->bvh_stack = max_stack;
    c->n_render_nodes = dn.size();
    const pt_bvh_node* N = s->nodes;
    for (int k = 0; k < 3; ++k) {
      c->root_lo[k] = round_down(N[0].bb_min[k]);
      c->root_hi[k] = round_up(N[0].bb_max[k]);
      c->root_lo_d[k] = N[0].bb_min[k];
      c->root_hi_d[k] = N[0].bb_max[k];
    }
  } else {
    int rc = build_gpu_bvh(c, s);
    if (rc) return rc;
  }
  HIPCHK(hipMemcpy(c->bsdfs.p, bs.data(), bs.size() * sizeof(DBsdf), hipMemcpyHostToDevice));
  if (!ls.empty()) HIPCHK(hipMemcpy(c->lights.p, ls.data(), ls.size() * sizeof(DLight), hipMemcpyHostToDevice));
  c->env_w = n_env ? s->env_width : 0;
  c->env_h = n_env ? s->env_height : 0;
  if (n_env) {
    HIPCHK(c->env_tex.reserve(env.tex.size()));
    HIPCHK(c->env_ptheta.reserve(env.p_theta.size()));
    HIPCHK(c->env_pphi.reserve(env.p_phi.size()));
    HIPCHK(c->env_pdf.reserve(env.p_theta_phi.size()));
    HIPCHK(hipMemcpy(c->env_tex.p, env.tex.data(), env.tex.size() * sizeof(float4), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->env_ptheta.p, env.p_theta.data(), env.p_theta.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->env_pphi.p, env.p_phi.data(), env.p_phi.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->env_pdf.p, env.p_theta_phi.data(), env.p_theta_phi.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(c->env_rtheta.reserve(env.r_theta.size()));
    HIPCHK(c->env_rphi.reserve(env.r_phi.size()));
    HIPCHK(hipMemcpy(c->env_rtheta.p, env.r_theta.data(), env.r_theta.size() * sizeof(EnvRec), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->env_rphi.p, env.r_phi.data(), env.r_phi.size() * sizeof(EnvRec), hipMemcpyHostToDevice));
  }
  c->n_lights = (int)ls.size();
  c->n_bsdfs = (int)bs.size();
  c->n_prims = s->n_prims;
  c->tri_only = std::all_of(s->prim_type, s->prim_type + s->n_prims, [](int t) { return t == PT_PRIM_TRIANGLE; });
  c->have_scene = true;
  return PT_OK;
}


int pt_upload_scene(pt_ctx* c, const pt_scene* s) { return upload_impl(c, s, false); }

int pt_upload_scene_lbvh(pt_ctx* c, const pt_scene* s) { return upload_impl(c, s, true); }

int pt_set_camera(pt_ctx* c, const pt_camera* cam) {
  if (!c || !cam) return fail(PT_E_INVALID, "pt_set_camera: NULL argument");
  if (int rc = tile_launch(c)) return rc;
  if (!(cam->screen_dist > 0) || !(cam->screen_w > 0) || !(cam->screen_h > 0))
    return fail(PT_E_INVALID, "pt_set_camera: non-positive screen size/distance");
  c->cam = *cam;
  c->have_cam = true;
  return PT_OK;
}

int pt_set_params(pt_ctx* c, const pt_params* p) {
  if (!c || !p) return fail(PT_E_INVALID, "pt_set_params: NULL argument");
  if (int rc = tile_launch(c)) return rc;
  if (p->width <= 0 || p->height <= 0 || p->spp <= 0 || p->max_depth < 0 || p->ns_area_light <= 0)
    return fail(PT_E_INVALID, "pt_set_params: width/height/spp/ns_area_light must be positive, max_depth >= 0");
  if (p->max_depth > 254 || p->ns_area_light > 255)  // packed in 8 bits each in the kernel's path state
    return fail(PT_E_INVALID, "pt_set_params: max_depth must be <= 254 and ns_area_light <= 255");
  if ((int64_t)p->width * p->height > (int64_t)1 << 30) return fail(PT_E_INVALID, "pt_set_params: frame too large");
  if (p->width > 65535 || p->height > 65535)  // pixel coordinates are packed in 16 bits each in the kernel
    return fail(PT_E_INVALID, "pt_set_params: width and height must be <= 65535");
  c->params = *p;
  c->have_params = true;
  return PT_OK;
}

static int build_tiles(pt_ctx* c, const pt_tile* tiles, int32_t n, std::vector<int4>& out) {
  const int W = c->params.width, H = c->params.height;
  for (int32_t i = 0; i < n; ++i) {
    const pt_tile& t = tiles[i];
    if (t.w < 0 || t.h < 0) return fail(PT_E_INVALID, "pt_render_tiles: negative tile size");
    int x0 = std::max(0, t.x), y0 = std::max(0, t.y);
    int x1 = std::min(W, t.x + t.w), y1 = std::min(H, t.y + t.h);  // raytrace_tile clamps (pathtracer.cpp:594-595)
    for (int y = y0; y < y1; y += 32)
      for (int x = x0; x < x1; x += 32) out.push_back(make_int4(x, y, std::min(32, x1 - x), std::min(32, y1 - y)));
  }
  return PT_OK;
}

// Conservative pixel rectangle covering the scene box as seen by the camera.
// Camera::generate_ray (camera.cpp:113-129) sends every ray of every pixel
// through the pinhole `pos` with direction c2w * ((fx-.5)W/d, (fy-.5)H/d, -1);
// a box entirely in front of the pinhole projects inside the rectangle of its
// 8 projected corners.  Rays start one unit BEHIND the pinhole, so the
// rectangle is only used when the box lies in front of the pinhole plane;
// otherwise (false) no pixel can be culled.  One pixel of margin absorbs
// rounding.  r = (x0, y0, x1, y1), inclusive, NOT clamped to the frame.
static bool footprint_rect(const pt_ctx* c, int W, int H, int r[4]) {
  const pt_camera& cam = c->cam;
  for (int i = 0; i < 3; ++i)  // coordinates by dot products need an orthonormal c2w
    for (int j = 0; j < 3; ++j) {
      double dp = 0;
      for (int k = 0; k < 3; ++k) dp += cam.c2w[3 * k + i] * cam.c2w[3 * k + j];
      if (std::fabs(dp - (i == j ? 1.0 : 0.0)) > 1e-9) return false;
    }
  double ax = cam.screen_w / cam.screen_dist, ay = cam.screen_h / cam.screen_dist;
  double x0 = 1e300, x1 = -1e300, y0 = 1e300, y1 = -1e300;
  for (int k = 0; k < 8; ++k) {
    double X[3] = {(k & 1) ? c->root_hi_d[0] : c->root_lo_d[0], (k & 2) ? c->root_hi_d[1] : c->root_lo_d[1],
                   (k & 4) ? c->root_hi_d[2] : c->root_lo_d[2]};
    double v[3] = {X[0] - cam.pos[0], X[1] - cam.pos[1], X[2] - cam.pos[2]};
    double cx = 0, cy = 0, cz = 0;  // coordinates along the c2w columns
    for (int i = 0; i < 3; ++i) {
      cx += v[i] * cam.c2w[3 * i + 0];
      cy += v[i] * cam.c2w[3 * i + 1];
      cz += v[i] * cam.c2w[3 * i + 2];
    }
    double depth = -cz;  // the view direction is -column 2
    if (!(depth > 1e-6 * (std::fabs(cx) + std::fabs(cy) + 1.0))) return false;  // behind / at the pinhole plane
    double fx = 0.5 + cx / depth / ax, fy = 0.5 + cy / depth / ay;
    x0 = std::min(x0, fx * W);
    x1 = std::max(x1, fx * W);
    y0 = std::min(y0, fy * H);
    y1 = std::max(y1, fy * H);
  }
  // pixel x covers [x, x+1) in fx*W
  r[0] = (int)std::max(-1.0, std::floor(x0) - 1);
  r[2] = (int)std::min((double)W, std::floor(x1) + 1);
  r[1] = (int)std::max(-1.0, std::floor(y0) - 1);
  r[3] = (int)std::min((double)H, std::floor(y1) + 1);
  return true;
}

// The culling rectangle: pixels outside [cull_x0, cull_x1] x [cull_y0,
// cull_y1] see no geometry (not traced, resolved to 0).
static void screen_footprint(const pt_ctx* c, KParams& P) {
  P.cull_x0 = 0;
  P.cull_y0 = 0;
  P.cull_x1 = P.W - 1;
  P.cull_y1 = P.H - 1;
  if (std::getenv("PT_NO_FOOTPRINT_CULL")) return;
  if (c->env_w > 0) return;  // rays that miss the scene see the environment map
  int r[4];
  if (!footprint_rect(c, P.W, P.H, r)) return;
  P.cull_x0 = r[0];
  P.cull_y0 = r[1];
  P.cull_x1 = r[2];
  P.cull_y1 = r[3];
}

// Pixels whose camera rays can reach the scene: the footprint's area inside
// the frame, or the whole frame with an environment light (misses see the
// map) or no footprint.  A property of the frame -- PT_NO_FOOTPRINT_CULL
// leaves it alone -- for the sample-group size.
static int64_t traced_px(const pt_ctx* c, int W, int H) {
  int r[4];
  if (c->env_w > 0 || !footprint_rect(c, W, H, r)) return (int64_t)W * H;
  const int64_t w = std::min(W - 1, r[2]) - std::max(0, r[0]) + 1, h = std::min(H - 1, r[3]) - std::max(0, r[1]) + 1;
  return std::max<int64_t>(0, w) * std::max<int64_t>(0, h);
}

// Sample groups of a pixel (KParams: n_groups groups of group_spp samples,
// the last one possibly short).  The grouping decides the float summation
// order of a pixel, so it is a function of the FRAME only -- its size, spp,
// the pixels its camera rays can reach, the environment light -- never of
// the launch's tile set, of a stats build or of the device: any split of a
// frame into tile launches (raytrace_tile calls, the multi-GPU shards) and
// any device (a CPX partition, fewer resident waves) sums every pixel in the
// same order.  The slots-per-lane rule below counts the lanes of a whole
// MI355X at the default occupancy (PT_GROUP_REF_LANES: 256 CUs x 20 waves x
// 64), not the running device's.
//  * group_spp: 4 (C4 +4%, framed C3 +2% over 2), 2 with an environment
//    light (C5 +2.3%, c5big +2.1%), halved until the traced samples make >= 24
//    work slots per resident lane: C3's footprint-culled frame gets 2 (+1.5%
//    pipelined, its lone launch 1.70 -> 1.44 ms: half the work in flight when
//    the queue runs dry), C1 / C2 get 1 (profiles/r4/ab_group_size.txt);
//  * (a tail of one-sample groups handed out last, to end the launch on short
//    work slots, measured -2% pipelined for +2% on a lone frame: DESIGN.md §4).
//  * `budget_waves` bounds the 32-bit slot indices: the largest grid any
//    launch of the frame may use (plain or stats build), so a frame that fits
//    one build fits the other.
static int group_size(int64_t traced, bool env, int spp, int64_t lanes, int64_t frame_blocks, int64_t budget_waves) {
  int gs = env ? PT_GROUP_SPP_ENV : PT_GROUP_SPP;
  while (gs > 1 && traced * ((spp + gs - 1) / gs) < lanes * PT_GROUP_MIN_SLOTS) gs /= 2;
  if (const char* g = std::getenv("PT_SAMPLE_GROUP")) {  // tuning knob
    int v = std::atoi(g);
    if (v > 0) gs = v;
  }
  gs = std::max(1, std::min(gs, spp));
  for (;;) {
    // 32-bit slot indices (they may overshoot by a static and a claimed
    // chunk per wave) and a group-sum budget of PT_GROUP_SUM_GIB per render
    // slot, for the whole frame's blocks (so every tile split gets the same
    // layout)
    const int64_t slots = frame_blocks * 64 * ((spp + gs - 1) / gs);
    if ((slots + 2 * budget_waves * PT_CHUNK_MAX < (int64_t)INT32_MAX && slots * PT_SUM_BYTES <= ((int64_t)PT_GROUP_SUM_GIB << 30)) ||
        gs >= spp)
      break;
    gs = std::min(spp, gs * 2);
  }
  return gs;
}

static int frames_that_fit(const pt_ctx* c, const std::vector<int4>& tl, int nf);

// One render: the render kernel on the slot's render stream, then the resolve
// on the caller's stream `s`, ordered after the render (see pt_ctx: the render
// pipeline).  (The resolve on the render stream instead measured one frame
// +0.03 ms: profiles/r5/ab_resolve_reset_stream.txt.)  `nf` > 1: a frame batch
// (pt_render_frames_device) -- nf frames of these tiles, frame f keyed by
// seeds[f] into outs[f], in ONE render launch (the MF kernel) and nf resolves;
// `seeds` null: the parameters' seed.
static int launch(pt_ctx* c, const std::vector<int4>& tl_in, float* const* outs, int nf, const uint32_t* seeds,
                  hipStream_t s, uint32_t flags) {
  const bool stats = (flags & (PT_FLAG_STATS | PT_FLAG_REF_COUNTS)) != 0;
  std::memset(&c->last, 0, sizeof(c->last));
  c->times_pending = false;
  if (tl_in.empty()) return PT_OK;
  // Large launches over trees larger than two XCD L2s render their tiles in
  // Z-order (the queue bands below then deal each XCD a compact region
  // rather than a strip of rows: C5 +2.5%, c5big +2.7%; C4's 4-MB tree,
  // without bands, -0.5% in Z-order, keeps the rows: profiles/r6/
  // ab_tile_zorder.txt).  Images are per
  // pixel and sample, identical in any order; packed outputs keep the
  // caller's tile index (tile_out).  PT_TILE_ZORDER=0/1 forces it (A/B, tests).
  std::vector<int4> tz;
  std::vector<int> tperm;
  {
    int64_t px = 0;
    int edge = 1;  // the tile edge: the largest tile's (clipped edge tiles are smaller)
    for (const int4& t : tl_in) {
      px += (int64_t)t.z * t.w;
      edge = std::max(edge, std::max(t.z, t.w));
    }
    bool z = tl_in.size() > 1 && px >= ((int64_t)1 << 20) &&
             (int64_t)c->n_render_nodes * 128 > ((int64_t)PT_BANDS_TREE_MIB << 20);
    if (const char* zo = std::getenv("PT_TILE_ZORDER")) z = tl_in.size() > 1 && std::atoi(zo) != 0;
    if (z) {
      std::vector<uint64_t> key(tl_in.size());
      for (size_t i = 0; i < tl_in.size(); ++i) {
        const uint64_t cx = (uint64_t)std::max(0, tl_in[i].x / edge), cy = (uint64_t)std::max(0, tl_in[i].y / edge);
        uint64_t k = 0;
        for (int b = 0; b < 21; ++b) k |= ((cx >> b) & 1ull) << (2 * b) | ((cy >> b) & 1ull) << (2 * b + 1);
        key[i] = k;
      }
      tperm.resize(tl_in.size());
      for (size_t i = 0; i < tperm.size(); ++i) tperm[i] = (int)i;
      std::stable_sort(tperm.begin(), tperm.end(), [&](int a, int b) { return key[a] < key[b]; });
      tz.resize(tl_in.size());
      for (size_t i = 0; i < tz.size(); ++i) tz[i] = tl_in[tperm[i]];
    }
  }
  const std::vector<int4>& tl = tperm.empty() ? tl_in : tz;
  c->last.tile_zorder = tperm.empty() ? 0 : 1;
  // PT_PIPELINE=0: every render on the caller's stream, one slot (A/B).  A
  // census launch (PT_CENSUS) writes its per-wave records into the one shared
  // trace area, so it never overlaps another launch: it runs unpipelined too.
  static const bool pipeline = (!std::getenv("PT_PIPELINE") || std::atoi(std::getenv("PT_PIPELINE")) != 0);
  const bool census_launch = std::getenv("PT_CENSUS") && !stats;
  const int depth = c->small_last ? pt_ctx::kSlots : pt_ctx::kSlotsLarge;
  const int slot = pipeline && !census_launch ? (int)(c->slot_rr++ % (uint64_t)depth) : 0;
  // A launch that finds every slot's last resolve complete has no frame to
  // overlap with: it runs on the caller's stream, with no cross-stream waits
  // in front of the render or between the render and the resolve (a lone
  // frame's wall clock; the slots still alternate).  Only hipErrorNotReady
  // means busy: any other result is a fault of an earlier render, reported
  // here instead of being absorbed into the choice.
  bool gpu_idle = true;  // no earlier render of this context still running or queued
  for (int k = 0; k < pt_ctx::kSlots && gpu_idle; ++k) {
    if (!c->ev_free[k]) continue;  // (a slot never used)
    const hipError_t q = hipEventQuery(c->ev_free[k]);
    if (q == hipErrorNotReady) {
      (void)hipGetLastError();  // (a not-ready query is no error of this launch)
      gpu_idle = false;
    } else if (q != hipSuccess) {
      return fail(PT_E_HIP, std::string("render: an earlier launch failed: ") + hipGetErrorString(q));
    }
  }
  const bool idle = pipeline && !census_launch && gpu_idle;
  if (!c->rstream[slot]) {  // a small launch's first use of slots 2 and 3
    HIPCHK(make_render_stream(&c->rstream[slot]));
    HIPCHK(hipEventCreateWithFlags(&c->ev_free[slot], hipEventDisableTiming));
    HIPCHK(hipEventRecord(c->ev_free[slot], c->stream));
  }
  hipStream_t rs = pipeline && !census_launch && !idle ? c->rstream[slot] : s;
  // the slot's device state is free once the previous resolve that read it ran
  if (!idle) HIPCHK(hipStreamWaitEvent(rs, c->ev_free[slot], 0));
  // the tile list rarely changes between frames: upload it only when it does
  std::vector<int4>& th = c->tiles_host[slot];
  if (tl.size() != th.size() || std::memcmp(tl.data(), th.data(), tl.size() * sizeof(int4)) != 0) {
    th = tl;
    HIPCHK(c->tiles[slot].reserve(tl.size()));
    HIPCHK(hipMemcpyAsync(c->tiles[slot].p, th.data(), th.size() * sizeof(int4), hipMemcpyHostToDevice, rs));
  }
  // Queue heads: zeroed by the slot's previous resolve (a memset in front of the render is a dependent launch of its own, ~20 us
  // before the render kernel starts on a lone frame); a memset only when
  // that did not happen (first use, a launch that failed half-way)
  if (!c->counter_clean[slot])
    HIPCHK(hipMemsetAsync(c->counter[slot].p, 0, PT_QUEUE_WORDS * PT_QUEUE_HEADS * sizeof(uint32_t), rs));
  c->counter_clean[slot] = false;
  if (stats) {
    unsigned long long init[PT_STATS_SLOTS] = {0};
    init[21] = init[23] = init[25] = ~0ull;  // atomicMin slots
    HIPCHK(hipMemcpyAsync(c->stats.p, init, sizeof(init), hipMemcpyHostToDevice, rs));
    HIPCHK(hipStreamSynchronize(rs));  // `init` is a stack array
  }
  KParams P;
  std::memset(&P, 0, sizeof(P));
  for (int k = 0; k < 3; ++k) {
    P.cam_pos[k] = (float)c->cam.pos[k];
    P.c2w_col0[k] = (float)c->cam.c2w[3 * k + 0];
    P.c2w_col1[k] = (float)c->cam.c2w[3 * k + 1];
    P.c2w_col2[k] = (float)c->cam.c2w[3 * k + 2];
  }
  P.cam_ax = (float)(c->cam.screen_w / c->cam.screen_dist);
  P.cam_ay = (float)(c->cam.screen_h / c->cam.screen_dist);
  P.W = c->params.width;
  P.H = c->params.height;
  P.inv_w = 1.0f / (float)P.W;
  P.inv_h = 1.0f / (float)P.H;
  P.spp = c->params.spp;
  P.max_depth = c->params.max_depth;
  P.ns_area = c->params.ns_area_light;
  P.nls_scale = (float)(1.0 / (double)P.ns_area);
  P.seed = seeds ? seeds[0] : c->params.seed;
  P.sample_base = c->params.sample_base;
  P.n_frames = nf;
  for (int f = 0; f < PT_MAX_FRAMES; ++f) P.seeds[f] = seeds && f < nf ? seeds[f] : P.seed;
  P.n_lights = c->n_lights;
  P.n_bsdfs = c->n_bsdfs;
  P.n_tiles = (int)tl.size();
  P.nodes = c->nodes.p;
  P.nodes2 = c->nodes2.p;
  P.prims = c->prims.p;
  P.norms = c->norms.p;
  if ((flags & PT_FLAG_REF_COUNTS) && c->prims_ref.p) {  // nodes2 indexes the caller's order
    P.prims = c->prims_ref.p;
    P.norms = c->norms_ref.p;
  }
  P.bsdfs = c->bsdfs.p;
  P.lights = c->lights.p;
  P.env_w = c->env_w;
  P.env_h = c->env_h;
  P.env_tex = c->env_tex.p;
  P.env_ptheta = c->env_ptheta.p;
  P.env_pphi = c->env_pphi.p;
  P.env_pdf = c->env_pdf.p;
  P.env_rtheta = c->env_rtheta.p;
  P.env_rphi = c->env_rphi.p;
  P.tiles = c->tiles[slot].p;
  P.tile_out = nullptr;
  if (!tperm.empty() && (flags & (PT_FLAG_PACKED | PT_FLAG_PACKED16))) {
    std::vector<int>& oh = c->tout_host[slot];
    if (oh != tperm) {
      oh = tperm;
      HIPCHK(c->tout[slot].reserve(oh.size()));
      HIPCHK(hipMemcpyAsync(c->tout[slot].p, oh.data(), oh.size() * sizeof(int), hipMemcpyHostToDevice, rs));
    }
    P.tile_out = c->tout[slot].p;
  }
  P.out = outs[0];
  P.packed = (flags & PT_FLAG_PACKED16) ? 16 : (flags & PT_FLAG_PACKED) ? 32 : 0;
  P.work_counter = c->counter[slot].p;
  P.stats = c->stats.p;
  P.dbg_pix = -1;
  for (int k = 0; k < 3; ++k) {
    P.root_lo[k] = c->root_lo[k];
    P.root_hi[k] = c->root_hi[k];
  }
  screen_footprint(c, P);
  c->last.footprint[0] = std::max(0, P.cull_x0);
  c->last.footprint[1] = std::max(0, P.cull_y0);
  c->last.footprint[2] = std::min(P.W - 1, P.cull_x1);
  c->last.footprint[3] = std::min(P.H - 1, P.cull_y1);
  if (c->last.footprint[2] < c->last.footprint[0] || c->last.footprint[3] < c->last.footprint[1]) {
    c->last.footprint[0] = c->last.footprint[1] = 0;  // nothing visible: the empty rectangle
    c->last.footprint[2] = c->last.footprint[3] = -1;
  }
  P.shade_batch = c->env_w > 0 ? PT_SHADE_BATCH_ENV : PT_SHADE_BATCH;
  P.leaf_weight = c->env_w > 0 ? PT_LEAF_WEIGHT_ENV : PT_LEAF_WEIGHT;
  if (const char* lw = std::getenv("PT_LEAF_WEIGHT")) {  // tuning knob
    int v = std::atoi(lw);
    if (v >= 1) P.leaf_weight = v;
  }
  P.census = census_launch ? 1 : 0;  // diagnostics (tools/wave_trace.py --census)
  // triangle-only scenes take the render kernel without the sphere test
  // (branch-free leaf steps); PT_NO_TRI_ONLY forces the mixed one (A/B, tests)
  P.tri_only = c->tri_only && !std::getenv("PT_NO_TRI_ONLY") ? 1 : 0;
  // drain helpers; PT_NO_HELPERS turns them off (A/B, tests)
  P.helpers = std::getenv("PT_NO_HELPERS") ? 0 : 1;
  P.drain_div = 0;
  if (const char* dd = std::getenv("PT_DRAIN_DIV")) {  // tuning knob
    int v = std::atoi(dd);
    if (v >= 0 && v <= 64) P.drain_div = v;
  }
  if (const char* sb = std::getenv("PT_SHADE_BATCH")) {  // tuning knob
    int v = std::atoi(sb);
    if (v >= 1 && v <= 64) P.shade_batch = v;
  }
  if (const char* dp = std::getenv("PT_DEBUG_PIXEL")) {  // diagnostics only
    int dx = -1, dy = -1;
    if (std::sscanf(dp, "%d,%d", &dx, &dy) == 2 && dx >= 0 && dy >= 0 && dx < P.W && dy < P.H) P.dbg_pix = dx + dy * P.W;
  }
  // Render blocks: <= 8x8 rectangles of each tile clipped to the footprint,
  // tile by tile (tb0[i] = the first block of tile i, for the resolve).
  std::vector<int4> bl;
  std::vector<int> tb0;
  tb0.reserve(tl.size() + 1);
  int64_t px_in = 0, px_all = 0;
  for (const int4& t : tl) {
    tb0.push_back((int)bl.size());
    px_all += (int64_t)t.z * t.w;
    int x0 = std::max(t.x, P.cull_x0), x1 = std::min(t.x + t.z - 1, P.cull_x1);
    int y0 = std::max(t.y, P.cull_y0), y1 = std::min(t.y + t.w - 1, P.cull_y1);
    for (int by = y0; by <= y1; by += 8)
      for (int bx = x0; bx <= x1; bx += 8) {
        bl.push_back(make_int4(bx, by, std::min(8, x1 - bx + 1), std::min(8, y1 - by + 1)));
        px_in += (int64_t)bl.back().z * bl.back().w;
      }
  }
  tb0.push_back((int)bl.size());
  c->culled_px = px_all - px_in;
  std::vector<int4>& bh = c->blocks_host[slot];
  if (!c->blocks[slot].p) HIPCHK(c->blocks[slot].reserve(1));  // never a null block list (a launch may cull every block)
  if (bl.size() != bh.size() || std::memcmp(bl.data(), bh.data(), bl.size() * sizeof(int4)) != 0) {
    bh = bl;
    HIPCHK(c->blocks[slot].reserve(bl.size()));
    if (!bh.empty())
      HIPCHK(hipMemcpyAsync(c->blocks[slot].p, bh.data(), bh.size() * sizeof(int4), hipMemcpyHostToDevice, rs));
  }
  P.blocks = c->blocks[slot].p;
  P.n_blocks = (int)bl.size();
  std::vector<int>& th0 = c->tblock0_host[slot];
  if (tb0 != th0) {
    th0 = tb0;
    HIPCHK(c->tblock0[slot].reserve(tb0.size()));
    HIPCHK(hipMemcpyAsync(c->tblock0[slot].p, th0.data(), th0.size() * sizeof(int), hipMemcpyHostToDevice, rs));
  }
  P.tile_block0 = c->tblock0[slot].p;
  // Work slots are (pixel, group of group_spp samples): small enough that
  // the dynamic queue balances the waves (a whole pixel per slot left the
  // launch waiting on a few waves holding 64-sample pixels).
  // the launch fills the GPU with the resident waves of the kernel variant it
  // runs (environment light / global tables; the STATS build for counters)
  const bool gtab = c->n_bsdfs > PT_LDS_BSDFS || c->n_lights > PT_LDS_LIGHTS || std::getenv("PT_FORCE_GLOBAL_TABLES");
  int64_t want = stats ? c->grid_stats
                       : (int64_t)std::max(8, c->bpc_variant[(c->env_w > 0 ? 2 : 0) + (gtab ? 1 : 0)]) * c->n_cu;
  if (const char* g = std::getenv("PT_WAVES_PER_CU")) {  // tuning knob
    int w = std::atoi(g);
    if (w > 0) want = (int64_t)w * c->n_cu;
  }
  const int64_t want_plain = std::getenv("PT_WAVES_PER_CU") ? want : c->grid_plain;
  const int64_t frame_blocks = (int64_t)((P.W + 7) / 8) * ((P.H + 7) / 8);
  const int64_t budget_waves = std::max({want, want_plain, (int64_t)c->grid_stats});
  P.group_spp = group_size(traced_px(c, P.W, P.H), c->env_w > 0, P.spp, (int64_t)PT_GROUP_REF_LANES, frame_blocks,
                           budget_waves);
  P.n_groups = (P.spp + P.group_spp - 1) / P.group_spp;
  const int64_t frame_slots = (int64_t)bl.size() * 64 * P.n_groups;
  const int64_t slots = frame_slots * nf;  // (a frame batch: every frame's slots, frame after frame)
  P.frame_slots = (uint32_t)frame_slots;
  pt_fastdiv_init((uint32_t)std::max<int64_t>(frame_slots, 1), &P.frm_m, &P.frm_sh);
  // (slot indices reach past the end by up to a static chunk plus a claimed one per wave)
  if (slots + 2 * want * PT_CHUNK_MAX >= (int64_t)INT32_MAX) return fail(PT_E_INVALID, "frame too large for one launch");
  // Small launches: at most PT_SMALL_SLOTS work slots per lane of the whole
  // resident grid (a strong split's share of the C3 frame: 12.8 at N = 2,
  // 3.2 at N = 8; the whole C3 frame has 25.6).  Each lane then renders only
  // a few slots, so a wave's slowest lane -- not the work -- sets the launch's
  // time.  They claim 64 slots at a time (one per lane: no wave holds two
  // while others have none), and when queued behind other frames they run on
  // half the resident grid with up to kSlots frames in flight (more slots per
  // lane per launch, the next frames filling each launch's tail).  Measured
  // on the split's share (one-GPU emulation, profiles/r6/ab_small_launch*.txt):
  // N = 8 0.38 -> 0.22 ms per frame, N = 4 0.51 -> 0.39, N = 2 0.75 -> 0.66.
  // Neither the grid nor the claim changes a value (the sample grouping is
  // a function of the frame).  PT_SMALL_LAUNCH=0 turns it off.
  static const bool small_on = !std::getenv("PT_SMALL_LAUNCH") || std::atoi(std::getenv("PT_SMALL_LAUNCH")) != 0;
  const bool small = small_on && pipeline && !census_launch && !stats &&
                     slots <= (int64_t)PT_SMALL_SLOTS * c->grid_plain * PT_BLOCK;
  if (!stats) c->small_last = small;
  if (small && !gpu_idle && !std::getenv("PT_WAVES_PER_CU")) want = std::max<int64_t>(c->n_cu, want / 2);
  pt_fastdiv_init((uint32_t)P.n_groups, &P.grp_m, &P.grp_sh);
  // queue claims: bigger for frames with many slots per lane (fewer atomics
  // on the heads; a lone small frame's drain prefers the smaller claim)
  // and for a frame queued behind another in the render pipeline
  // (profiles/r5/ab_chunk_busy.txt): its drain overlaps the previous frame's -- the
  // throughput case -- while a frame launched on an idle GPU, or with the
  // pipeline off (PT_PIPELINE=0: no two launches overlap), is the latency
  // case, whose end the smaller claim shortens
  // (C3: 256-slot claims +2.9% pipelined, lone launch +9%:
  // profiles/r5/ab_chunk_heads.txt).  A claim size never changes a value.
  const bool big_frame = slots >= (int64_t)PT_CHUNK_BIG_SLOTS * want_plain * PT_BLOCK;
  P.chunk = small ? PT_BLOCK
          : big_frame || (pipeline && !census_launch && !gpu_idle) ? PT_CHUNK_MAX
                                                                   : PT_CHUNK;
  // large frames claim PT_CHUNK_BIG (512) where the slot indices and the
  // one-block-per-chunk rule allow it: half the atomics again (C5 +1.0%, C4
  // +0.7%; C3's queued frames lose 7% at 512: profiles/r5/ab_chunk512.txt)
  if (big_frame && slots + 2 * want * PT_CHUNK_BIG < (int64_t)INT32_MAX && (64 * P.n_groups) % PT_CHUNK_BIG == 0)
    P.chunk = PT_CHUNK_BIG;
  if (const char* cs = std::getenv("PT_CHUNK_SLOTS")) {  // tuning knob (64..PT_CHUNK_BIG, a multiple of 64)
    const int v = std::atoi(cs);
    if (v >= 64 && v <= PT_CHUNK_BIG && v % 64 == 0 && slots + 2 * want * v < (int64_t)INT32_MAX) P.chunk = v;
  }
  // Large frames (PT_CHUNK_BIG_SLOTS slots per lane and more) over trees
  // larger than two XCD L2s (4 MB each): each queue head deals a contiguous
  // band of the frame, so an XCD's waves share BVH nodes in its L2 (C5's 17-MB
  // tree +1.8%, c5big's 68-MB +1.8%); C4's 4-MB tree loses 1.2% to the bands'
  // uneven ends, and a small frame keeps the interleaved sweep, whose heads
  // run dry together (C3 -5.5%, its lone launch +12%): profiles/r5/ab_bands*.txt.
  // PT_QUEUE_BANDS=0/1 forces it (A/B, tests).
  P.qbands = big_frame && (int64_t)c->n_render_nodes * 128 > ((int64_t)PT_BANDS_TREE_MIB << 20) ? 1 : 0;
  if (const char* qb = std::getenv("PT_QUEUE_BANDS")) P.qbands = std::atoi(qb) != 0 ? 1 : 0;
  P.sblocks = (64 * P.n_groups) % P.chunk == 0 ? 1 : 0;  // every (aligned) chunk inside one block
  // group sums: 12 B per work slot of THIS launch (a rank's share of a split
  // frame holds only its own blocks' sums)
  if (nf > 1) {
    // a frame batch: every render slot's group sums sized at once for the
    // largest batch of this tile set, and its spill area for the whole grid
    // (growing a buffer later synchronises the device -- inside the caller's
    // back-to-back frames)
    const size_t cap = (size_t)std::max<int64_t>(frame_slots, 1) * 3 *
                       (size_t)std::max(nf, frames_that_fit(c, tl, PT_MAX_FRAMES));
    for (int k = 0; k < pt_ctx::kSlots; ++k) {
      HIPCHK(c->partial[k].reserve(cap));
      if (c->bvh_stack > PT_STACK)
        HIPCHK(c->spill[k].reserve((size_t)(c->bvh_stack - PT_STACK) * std::max<int64_t>(want, c->grid_plain) * PT_BLOCK));
    }
  }
  HIPCHK(c->partial[slot].reserve((size_t)std::max<int64_t>(slots, 1) * 3));
  P.partial = c->partial[slot].p;
  c->last.partial_bytes = slots * PT_SUM_BYTES;
  auto log2_exact = [](int v) {  // log2(v) for a power of two, else -1
    int k = 0;
    while ((1 << k) < v && k < 30) ++k;
    return (1 << k) == v ? k : -1;
  };
  P.group_shift = log2_exact(P.group_spp);
  int64_t max_grid = std::max<int64_t>(1, (slots + PT_BLOCK - 1) / PT_BLOCK);
  int grid = (int)std::min<int64_t>(want, max_grid);
  if ((stats || P.census) && (size_t)grid * PT_WAVE_TRACE + PT_STATS_SLOTS > c->stats.n)
    grid = (int)((c->stats.n - PT_STATS_SLOTS) / PT_WAVE_TRACE);
  grid = std::max(1, grid);
  if (P.census)  // (a build without -DPT_CENSUS=1 leaves the drain fields 0)
    HIPCHK(hipMemsetAsync(c->stats.p + PT_STATS_SLOTS, 0, (size_t)grid * PT_WAVE_TRACE * 8, rs));
  P.stack_spill = nullptr;
  if (c->bvh_stack > PT_STACK) {  // worst-case depth beyond the LDS stack
    HIPCHK(c->spill[slot].reserve((size_t)(c->bvh_stack - PT_STACK) * grid * PT_BLOCK));
    P.stack_spill = c->spill[slot].p;
  }
  {
    hipEvent_t* tri = c->ev[c->n_launches % pt_ctx::kRing];
    c->ev0 = tri[0];
    c->ev1 = tri[1];
    c->ev2 = tri[2];
    ++c->n_launches;
  }
  HIPCHK(hipEventRecord(c->ev0, rs));
  HIPCHK(ptk_launch_render(&P, grid, stats, (flags & PT_FLAG_REF_COUNTS) != 0, rs));
  HIPCHK(hipEventRecord(c->ev1, rs));
  if (rs != s) HIPCHK(hipStreamWaitEvent(s, c->ev1, 0));  // the resolve reads the finished group sums
  for (int f = 0; f < nf; ++f) {  // (a frame batch: frame f's sums follow frame f - 1's)
    KParams Pf = P;
    Pf.partial = P.partial + 3 * (size_t)f * (size_t)frame_slots;
    Pf.out = outs[f];
    HIPCHK(ptk_launch_resolve(&Pf, s));
  }
  c->counter_clean[slot] = true;  // (the resolve zeroed the slot's queue heads)
  HIPCHK(hipEventRecord(c->ev2, s));
  HIPCHK(hipEventRecord(c->ev_free[slot], s));
  c->census_valid = P.census != 0;
  c->last.grid_blocks = grid;
  c->last.group_spp = P.group_spp;
  c->last.blocks_per_cu = (int32_t)(want / std::max(1, c->n_cu));
  int64_t px = 0;
  for (const int4& t : tl) px += (int64_t)t.z * t.w;
  c->last.pixels = px;
  c->last.bvh_stack = c->bvh_stack;
  c->last.bvh_nodes = (int64_t)c->n_render_nodes;
  c->last.samples = px * c->params.spp;
  c->last.frames_per_launch = nf;
  return PT_OK;
}

// The last launch's kernel / resolve times (waits for its events).
static int settle_times(pt_ctx* c) {
  if (!c->times_pending) return PT_OK;
  HIPCHK(hipEventSynchronize(c->ev2));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
  c->last.last_ms = ms;
  HIPCHK(hipEventElapsedTime(&ms, c->ev1, c->ev2));
  c->last.resolve_ms = ms;
  c->times_pending = false;
  return PT_OK;
}

// After a launch: counters (and times) of a stats launch now; a plain device
// launch stays asynchronous, its times are read when asked for.
static int finish_stats(pt_ctx* c, hipStream_t s, uint32_t flags, bool sync) {
  if (c->last.grid_blocks == 0) return PT_OK;  // nothing was launched
  c->times_pending = true;
  const bool counters = (flags & (PT_FLAG_STATS | PT_FLAG_REF_COUNTS)) != 0;
  if (!sync && !counters) return PT_OK;
  HIPCHK(hipStreamSynchronize(s));
  int rc = settle_times(c);
  if (rc) return rc;
  if (counters) {
    unsigned long long v[PT_STATS_SLOTS] = {0};
    HIPCHK(hipMemcpy(v, c->stats.p, sizeof(v), hipMemcpyDeviceToHost));
    c->last.camera_rays = (int64_t)v[0];
    c->last.bounce_rays = (int64_t)v[1];
    c->last.shadow_rays = (int64_t)v[2];
    c->last.node_visits = (int64_t)v[3];
    c->last.tri_tests = (int64_t)v[4];
    c->last.sphere_tests = (int64_t)v[5];
    c->last.ext_hits = (int64_t)v[6];
    c->last.wave_trav_steps = (int64_t)v[7];
    c->last.wave_rounds = (int64_t)v[8];
    c->last.culled_samples = c->culled_px * c->params.spp;
    c->last.leaf_steps = (int64_t)v[9];
    c->last.queue_atomics = (int64_t)v[10];
    c->last.shade_clocks = (int64_t)v[11];
    c->last.trav_clocks = (int64_t)v[12];
    c->last.max_wave_clocks = (int64_t)v[13];
    c->last.wave_wall_sum = (int64_t)v[14];
    c->last.wave_wall_max = (int64_t)v[15];
    c->last.hitshade_clocks = (int64_t)v[16];
    for (int k = 0; k < 4; ++k) c->last.section_clocks[k] = (int64_t)v[17 + k];
    for (int k = 0; k < 4; ++k) c->last.lane_iters[k] = (int64_t)v[27 + k];
    c->last.deep_stack_steps = (int64_t)v[31];
    for (int k = 0; k < 32; ++k) c->last.slot_latency_hist[k] = (int64_t)v[32 + k];
    for (int k = 0; k < 8; ++k) c->last.node_census[k] = (int64_t)v[64 + k];
    for (int k = 0; k < 3; ++k) c->last.wave_span[k] = (int64_t)(v[22 + k] - v[21]);
    for (int k = 0; k < 2; ++k) c->last.wave_span[3 + k] = v[25 + k] ? (int64_t)(v[25 + k] - v[21]) : -1;
    c->last.counters_valid = 1;
  }
  return PT_OK;
}

static int check_ready(pt_ctx* c) {
  if (!c) return fail(PT_E_INVALID, "NULL context");
  if (!c->have_scene || !c->have_cam || !c->have_params)
    return fail(PT_E_NOSCENE, "render before pt_upload_scene / pt_set_camera / pt_set_params");
  return PT_OK;
}

// True when no pixel belongs to two of the (clipped) tiles.
static bool tiles_disjoint(const std::vector<int4>& tl, size_t W, size_t H) {
  std::vector<uint8_t> seen(W * H, 0);
  for (const int4& t : tl)
    for (int y = t.y; y < t.y + t.w; ++y)
      for (int x = t.x; x < t.x + t.z; ++x) {
        uint8_t& v = seen[(size_t)y * W + (size_t)x];
        if (v) return false;
        v = 1;
      }
  return true;
}

int pt_render_tiles(pt_ctx* c, const pt_tile* tiles, int32_t n_tiles, float* hdr_out_host, uint32_t flags) {
  int rc = check_ready(c);
  if (rc) return rc;
  if ((rc = tile_launch(c))) return rc;  // earlier asynchronous tiles first (call order)
  if (n_tiles < 0 || (n_tiles > 0 && (!tiles || !hdr_out_host))) return fail(PT_E_INVALID, "pt_render_tiles: bad args");
  if (flags & (PT_FLAG_PACKED | PT_FLAG_PACKED16))
    return fail(PT_E_INVALID, "pt_render_tiles: packed output is for pt_render_tiles_device");
  HIPCHK(hipSetDevice(c->device));
  std::vector<int4> tl;
  if ((rc = build_tiles(c, tiles, n_tiles, tl))) return rc;
  const size_t W = (size_t)c->params.width, H = (size_t)c->params.height;
  HIPCHK(c->frame.reserve(W * H * 3));
  float* fr = c->frame.p;
  if ((rc = launch(c, tl, &fr, 1, nullptr, c->stream, flags))) return rc;
  // Copy back only the tiles' pixels (the caller's buffer is theirs outside
  // them); a call whose (clipped, disjoint) tiles cover the whole frame - the
  // whole-frame batch - is one contiguous copy.
  int64_t area = 0;
  for (const int4& t : tl) area += (int64_t)t.z * t.w;
  if (area == (int64_t)(W * H) && tiles_disjoint(tl, W, H)) {
    HIPCHK(hipMemcpyAsync(hdr_out_host, c->frame.p, W * H * 3 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  } else {
    for (const int4& t : tl) {
      size_t off = ((size_t)t.y * W + (size_t)t.x) * 3;
      HIPCHK(hipMemcpy2DAsync(hdr_out_host + off, W * 3 * sizeof(float), c->frame.p + off, W * 3 * sizeof(float),
                              (size_t)t.z * 3 * sizeof(float), (size_t)t.w, hipMemcpyDeviceToHost, c->stream));
    }
  }
  return finish_stats(c, c->stream, flags, true);
}

// PT_FLAG_PACKED / PT_FLAG_PACKED16: tile i -> packed slot i, so no clipping
// or splitting may renumber tiles: every tile 1..S x 1..S and inside the frame
static int check_packed(const pt_ctx* c, const pt_tile* tiles, int32_t n_tiles, uint32_t flags, const char* fn) {
  if (!(flags & (PT_FLAG_PACKED | PT_FLAG_PACKED16))) return PT_OK;
  const int S = (flags & PT_FLAG_PACKED16) ? 16 : 32;
  const int W = c->params.width, H = c->params.height;
  for (int32_t i = 0; i < n_tiles; ++i) {
    const pt_tile& t = tiles[i];
    if (t.w < 1 || t.h < 1 || t.w > S || t.h > S || t.x < 0 || t.y < 0 || t.x + t.w > W || t.y + t.h > H)
      return fail(PT_E_INVALID, std::string(fn) + ": packed output needs tiles of 1.." + std::to_string(S) + " x 1.." +
                                    std::to_string(S) + " inside the frame");
  }
  return PT_OK;
}

int pt_render_tiles_device(pt_ctx* c, const pt_tile* tiles, int32_t n_tiles, float* hdr_out_dev, void* stream,
                           uint32_t flags) {
  int rc = check_ready(c);
  if (rc) return rc;
  if ((rc = tile_launch(c))) return rc;
  if (n_tiles < 0 || (n_tiles > 0 && (!tiles || !hdr_out_dev)))
    return fail(PT_E_INVALID, "pt_render_tiles_device: bad args");
  HIPCHK(hipSetDevice(c->device));
  std::vector<int4> tl;
  if ((rc = build_tiles(c, tiles, n_tiles, tl))) return rc;
  if (int rc2 = check_packed(c, tiles, n_tiles, flags, "pt_render_tiles_device")) return rc2;
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  if ((rc = launch(c, tl, &hdr_out_dev, 1, nullptr, s, flags))) return rc;
  return finish_stats(c, s, flags, false);
}

// Frames of the tile set `tl` one launch of a frame batch takes.  A frame
// with more than PT_BATCH_SLOTS work slots per lane of a whole MI355X renders
// alone: it fills the GPU by itself, and batching measured slower there (C4
// -4.7%; C3's 25.6 slots per lane +2%, its strong split's shares +15..+45%:
// profiles/r6/ab_frame_batch.txt).  Otherwise as many as keep the work-slot
// indices (with the claims' overshoot, a grid of up to 40 waves per CU) 32-bit
// and the group sums within PT_GROUP_SUM_GIB.  The blocks are the launch's
// own (the tiles' 8x8 blocks inside the scene's screen footprint).
static int frames_that_fit(const pt_ctx* c, const std::vector<int4>& tl, int nf) {
  const int W = c->params.width, H = c->params.height;
  KParams fp;
  std::memset(&fp, 0, sizeof(fp));
  fp.W = W;
  fp.H = H;
  screen_footprint(c, fp);
  int64_t blocks = 0;
  for (const int4& t : tl) {
    const int x0 = std::max(t.x, fp.cull_x0), x1 = std::min(t.x + t.z - 1, fp.cull_x1);
    const int y0 = std::max(t.y, fp.cull_y0), y1 = std::min(t.y + t.w - 1, fp.cull_y1);
    if (x1 >= x0 && y1 >= y0) blocks += (int64_t)((x1 - x0 + 8) / 8) * ((y1 - y0 + 8) / 8);
  }
  const int64_t frame_blocks = (int64_t)((W + 7) / 8) * ((H + 7) / 8);
  const int64_t waves = std::max<int64_t>({(int64_t)c->grid_plain, (int64_t)c->grid_stats, (int64_t)40 * c->n_cu});
  const int gs = group_size(traced_px(c, W, H), c->env_w > 0, c->params.spp, (int64_t)PT_GROUP_REF_LANES,
                            frame_blocks, waves);
  const int64_t per = blocks * 64 * ((c->params.spp + gs - 1) / gs);
  if (per > (int64_t)PT_BATCH_SLOTS * PT_GROUP_REF_LANES) return 1;
  while (nf > 1 && (per * nf + 2 * waves * PT_CHUNK_BIG >= (int64_t)INT32_MAX ||
                    per * nf * PT_SUM_BYTES > ((int64_t)PT_GROUP_SUM_GIB << 30)))
    --nf;
  return nf;
}

int pt_render_frames_device(pt_ctx* c, const pt_tile* tiles, int32_t n_tiles, int32_t n_frames, const uint32_t* seeds,
                            float* const* hdr_outs_dev, void* stream, uint32_t flags) {
  int rc = check_ready(c);
  if (rc) return rc;
  if ((rc = tile_launch(c))) return rc;
  if (n_frames < 1 || n_frames > PT_MAX_FRAMES || !seeds || !hdr_outs_dev || n_tiles < 0 || (n_tiles > 0 && !tiles))
    return fail(PT_E_INVALID, "pt_render_frames_device: bad args (1 <= n_frames <= PT_MAX_FRAMES, seeds and outputs)");
  for (int32_t f = 0; f < n_frames; ++f)
    if (n_tiles > 0 && !hdr_outs_dev[f]) return fail(PT_E_INVALID, "pt_render_frames_device: NULL output");
  if (flags & (PT_FLAG_STATS | PT_FLAG_REF_COUNTS))
    return fail(PT_E_INVALID, "pt_render_frames_device: counters are per frame (pt_render_tiles_device)");
  HIPCHK(hipSetDevice(c->device));
  std::vector<int4> tl;
  if ((rc = build_tiles(c, tiles, n_tiles, tl))) return rc;
  if (int rc2 = check_packed(c, tiles, n_tiles, flags, "pt_render_frames_device")) return rc2;
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  // One launch for the batch in the plain common build; the environment-light
  // and global-table builds, diagnostics and PT_FRAME_BATCH=0 render the
  // frames one launch each (the same images)
  static const bool batch_on = !std::getenv("PT_FRAME_BATCH") || std::atoi(std::getenv("PT_FRAME_BATCH")) != 0;
  const bool gtab = c->n_bsdfs > PT_LDS_BSDFS || c->n_lights > PT_LDS_LIGHTS || std::getenv("PT_FORCE_GLOBAL_TABLES");
  const bool one = !batch_on || n_frames == 1 || c->env_w > 0 || gtab || std::getenv("PT_CENSUS") ||
                   std::getenv("PT_DEBUG_PIXEL");
  if (one) {
    for (int32_t f = 0; f < n_frames; ++f)
      if ((rc = launch(c, tl, &hdr_outs_dev[f], 1, &seeds[f], s, flags))) return rc;
  } else {
    // (frames beyond what one launch's slot indices and group sums hold go
    // into further batches)
    for (int32_t f = 0; f < n_frames;) {
      const int nf = frames_that_fit(c, tl, n_frames - f);
      if ((rc = launch(c, tl, hdr_outs_dev + f, nf, seeds + f, s, flags))) return rc;
      f += nf;
    }
  }
  return finish_stats(c, s, flags, false);
}

// ---- asynchronous one-tile seam
// Completion of one batch (on the completion thread, after the batch's event):
// the tiles' pixels go from the batch's stage into the caller's sampleBuffer
// and, as PathTracer::raytrace_tile does at its end (pathtracer.cpp:610),
// through toColor into its frameBuffer.
static void tile_complete(const pt_ctx::TileBatch* b) {
  for (const pt_ctx::TileJob& j : b->jobs) {
    for (int y = j.t.y; y < j.t.y + j.t.w; ++y) {
      const size_t dst = ((size_t)y * (size_t)b->W + (size_t)j.t.x) * 3;
      const size_t src = ((size_t)(y - b->y0) * (size_t)b->W + (size_t)j.t.x) * 3;
      std::memcpy(j.hdr + dst, b->stage + src, (size_t)j.t.z * 3 * sizeof(float));
    }
    if (j.rgba) (void)pt_to_color(j.hdr, b->W, b->H, j.t.x, j.t.y, j.t.x + j.t.z, j.t.y + j.t.w, j.rgba);
  }
}

// The completion thread: batches in launch order; each waits for its own
// event only, so completing batch k overlaps the render of batch k+1.
static void tile_worker(pt_ctx* c) {
  (void)hipSetDevice(c->device);
  for (;;) {
    pt_ctx::TileBatch* b = nullptr;
    {
      std::unique_lock<std::mutex> lk(c->tmu);
      c->tcv.wait(lk, [&] { return c->tstop || !c->tpending.empty(); });
      if (c->tpending.empty()) return;  // stopping, nothing left to complete
      b = c->tpending.front();
      c->tpending.pop_front();
    }
    const hipError_t e = hipEventSynchronize(b->ev);
    if (e == hipSuccess) tile_complete(b);
    std::lock_guard<std::mutex> lk(c->tmu);
    if (e != hipSuccess && c->terr == PT_OK) {
      c->terr = PT_E_HIP;
      c->terrmsg = std::string("tile completion: ") + hipGetErrorString(e);
    }
    b->jobs.clear();
    c->tfree.push_back(b);
    --c->tinflight;
    c->tcv.notify_all();
  }
}

static void tile_worker_stop(pt_ctx* c) {
  if (c->tworker.joinable()) {
    {
      std::lock_guard<std::mutex> lk(c->tmu);
      c->tstop = true;
    }
    c->tcv.notify_all();
    c->tworker.join();  // drains the pending batches first
  }
  for (auto* b : c->tfree) {
    if (b->stage) (void)hipHostFree(b->stage);
    if (b->ev) (void)hipEventDestroy(b->ev);
    delete b;
  }
  c->tfree.clear();
}

// A batch that could not be launched: its tiles are dropped, so the failure is
// also kept for the next pt_tile_finish (which would otherwise report PT_OK for
// tiles it never rendered), whoever called tile_launch.
static int tile_launch_failed(pt_ctx* c, int rc) {
  std::lock_guard<std::mutex> lk(c->tmu);
  if (c->terr == PT_OK) {
    c->terr = rc;
    c->terrmsg = std::string("tile launch: ") + pt_last_error();
  }
  return rc;
}

// Fault injection for the seam's error path (tests): PT_FAULT_TILE_LAUNCH=k
// at pt_create makes the context's k-th batch launch fail before it renders.
static bool tile_fault_injected(pt_ctx* c) {
  return c->fault_tile_launch > 0 && ++c->n_tile_launches == c->fault_tile_launch;
}

static int tile_launch_impl(pt_ctx* c);

// Renders the queued tiles as one launch (nothing queued: nothing to do).
static int tile_launch(pt_ctx* c) {
  if (!c || c->tq.empty()) return PT_OK;
  const int rc = tile_launch_impl(c);
  return rc ? tile_launch_failed(c, rc) : PT_OK;
}

static int tile_launch_impl(pt_ctx* c) {
  constexpr int kMaxBatchesInFlight = 8;  // bounds the pinned staging memory
  std::vector<pt_ctx::TileJob> jobs;
  jobs.swap(c->tq);
  if (tile_fault_injected(c)) return fail(PT_E_HIP, "pt_tile_submit: injected launch failure (PT_FAULT_TILE_LAUNCH)");
  HIPCHK(hipSetDevice(c->device));
  const size_t W = (size_t)c->params.width, H = (size_t)c->params.height;
  std::vector<int4> tl;
  for (const auto& j : jobs) tl.push_back(j.t);
  // the band of whole rows the batch's tiles span (a batch of the FIFO is a
  // few tile rows): one copy; pixels of the band outside the tiles land in
  // the stage only, never in the caller's buffers
  int y0 = (int)H, y1 = 0;
  for (const int4& t : tl) {
    y0 = std::min(y0, t.y);
    y1 = std::max(y1, t.y + t.w);
  }
  const size_t need = (size_t)(y1 - y0) * W * 3;
  pt_ctx::TileBatch* b = nullptr;
  {
    std::unique_lock<std::mutex> lk(c->tmu);
    if (!c->tworker.joinable()) {
      c->tstop = false;
      c->tworker = std::thread(tile_worker, c);
    }
    c->tcv.wait(lk, [&] { return !c->tfree.empty() || c->tinflight < kMaxBatchesInFlight; });
    if (!c->tfree.empty()) {
      b = c->tfree.back();
      c->tfree.pop_back();
    }
  }
  if (!b) b = new pt_ctx::TileBatch();
  auto give_back = [&] {
    std::lock_guard<std::mutex> lk(c->tmu);
    c->tfree.push_back(b);
  };
  if (b->cap < need) {
    if (b->stage) (void)hipHostFree(b->stage);
    b->stage = nullptr;
    b->cap = 0;
    if (hipHostMalloc((void**)&b->stage, need * sizeof(float), hipHostMallocDefault) != hipSuccess) {
      give_back();
      return fail(PT_E_HIP, "pt_tile_submit: pinned staging allocation failed");
    }
    b->cap = need;
  }
  if (!b->ev && hipEventCreateWithFlags(&b->ev, hipEventDisableTiming) != hipSuccess) {
    give_back();
    return fail(PT_E_HIP, "pt_tile_submit: event creation failed");
  }
  if (hipError_t e = c->frame.reserve(W * H * 3); e != hipSuccess) {
    give_back();
    return fail(PT_E_HIP, std::string("pt_tile_submit: ") + hipGetErrorString(e));
  }
  float* fr = c->frame.p;
  if (int rc = launch(c, tl, &fr, 1, nullptr, c->stream, 0)) {
    give_back();
    return rc;
  }
  hipError_t e = hipMemcpyAsync(b->stage, c->frame.p + (size_t)y0 * W * 3, need * sizeof(float),
                                hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipEventRecord(b->ev, c->stream);
  if (e != hipSuccess) {
    give_back();
    return fail(PT_E_HIP, std::string("pt_tile_submit: ") + hipGetErrorString(e));
  }
  b->jobs = std::move(jobs);
  b->y0 = y0;
  b->W = (int)W;
  b->H = (int)H;
  {
    std::lock_guard<std::mutex> lk(c->tmu);
    c->tpending.push_back(b);
    ++c->tinflight;
  }
  c->tcv.notify_all();
  return finish_stats(c, c->stream, 0, false);
}

int pt_tile_submit(pt_ctx* c, const pt_tile* tile, float* hdr_out_host, uint32_t* rgba_out_host) {
  int rc = check_ready(c);
  if (rc) return rc;
  if (!tile || !hdr_out_host) return fail(PT_E_INVALID, "pt_tile_submit: NULL tile or output");
  std::vector<int4> tl;
  if ((rc = build_tiles(c, tile, 1, tl))) return rc;  // clamped to the frame, <= 32 x 32 pieces
  for (const int4& t : tl) c->tq.push_back(pt_ctx::TileJob{t, hdr_out_host, rgba_out_host});
  if ((int)c->tq.size() >= c->tile_batch) return tile_launch(c);
  return PT_OK;
}

int pt_tile_finish(pt_ctx* c) {
  if (!c) return fail(PT_E_INVALID, "NULL context");
  // Whatever happens to the last launch, every batch already in flight is
  // waited for: the completion thread writes into the caller's buffers, which
  // the caller may free or reuse as soon as this returns.
  (void)tile_launch(c);  // (a failure is recorded in terr)
  int err = PT_OK;
  std::string msg;
  {
    std::unique_lock<std::mutex> lk(c->tmu);
    c->tcv.wait(lk, [&] { return c->tinflight == 0; });  // every batch copied and completed
    err = c->terr;
    msg = c->terrmsg;
    c->terr = PT_OK;
    c->terrmsg.clear();
  }
  if (err != PT_OK) return fail(err, msg);
  return PT_OK;
}

int pt_intersect(pt_ctx* c, int64_t n, const double* o, const double* d, const double* max_t, int32_t* hit, float* t,
                 int32_t* prim, int32_t* any_hit) {
  if (!c) return fail(PT_E_INVALID, "NULL context");
  if (!c->have_scene) return fail(PT_E_NOSCENE, "pt_intersect before pt_upload_scene");
  if (n < 0 || (n > 0 && (!o || !d || !max_t))) return fail(PT_E_INVALID, "pt_intersect: bad args");
  if (n == 0) return PT_OK;
  HIPCHK(hipSetDevice(c->device));
  std::vector<float> f((size_t)n * 7);
  for (int64_t i = 0; i < 3 * n; ++i) {
    f[(size_t)i] = (float)o[i];
    f[(size_t)(3 * n + i)] = (float)d[i];
  }
  for (int64_t i = 0; i < n; ++i) f[(size_t)(6 * n + i)] = (float)max_t[i];
  HIPCHK(c->q_f.reserve((size_t)n * 8));
  HIPCHK(c->q_i.reserve((size_t)n * 3));
  HIPCHK(hipMemcpyAsync(c->q_f.p, f.data(), f.size() * sizeof(float), hipMemcpyHostToDevice, c->stream));
  float* dt = c->q_f.p + 7 * n;
  int32_t* dh = c->q_i.p;
  int32_t* dp = c->q_i.p + n;
  int32_t* da = c->q_i.p + 2 * n;
  int* spill = nullptr;
  if (c->bvh_stack > PT_STACK) {
    HIPCHK(c->q_spill.reserve((size_t)(c->bvh_stack - PT_STACK) * (size_t)((n + PT_BLOCK - 1) / PT_BLOCK * PT_BLOCK)));
    spill = c->q_spill.p;
  }
  HIPCHK(ptk_launch_intersect(c->nodes.p, c->prims.p, c->q_f.p, c->q_f.p + 3 * n, c->q_f.p + 6 * n, n, dh, dt, dp, da,
                              spill, c->prim_map.p, c->stream));
  std::vector<int32_t> ib((size_t)n * 3);
  std::vector<float> tb((size_t)n);
  HIPCHK(hipMemcpyAsync(ib.data(), c->q_i.p, ib.size() * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(tb.data(), dt, tb.size() * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  for (int64_t i = 0; i < n; ++i) {
    if (hit) hit[i] = ib[(size_t)i];
    if (prim) prim[i] = ib[(size_t)(n + i)];
    if (any_hit) any_hit[i] = ib[(size_t)(2 * n + i)];
    if (t) t[i] = tb[(size_t)i];
  }
  return PT_OK;
}

// Host replay of the environment light's inverse-CDF searches (the kernel's
// record_lower_bound over the tables build_env_tables makes) against
// std::lower_bound, for n query pairs (u1, u2) in [0, 1): the row search over
// pTheta, then the column search over that row of pPhiGivenTheta, each checked
// for the index and the interpolation pair (prev, cur) the sampler reads.
int64_t pt_env_search_check(const float* rgb, int32_t width, int32_t height, int64_t n, const float* u1,
                            const float* u2, int64_t* long_windows) {
  if (!rgb || width <= 0 || height <= 0 || n < 0 || (n > 0 && (!u1 || !u2)))
    return fail(PT_E_INVALID, "pt_env_search_check: bad arguments");
  EnvTables t;
  build_env_tables(rgb, width, height, t);
  int64_t bad = 0, longw = 0;
  auto check = [&](const float* a, int len, const EnvRec* rec, float u) -> int {
    const float v = u * a[len - 1];
    const int k = std::min(PT_ENV_GUIDE - 1, std::max(0, (int)(u * (float)PT_ENV_GUIDE)));
    longw += rec[k].hi - rec[k].lo > 4;
    float prev = 0.f, cur = 0.f;
    const int got = record_lower_bound(a, v, u, rec, PT_ENV_GUIDE, prev, cur);
    const int want = (int)(std::lower_bound(a, a + len, v) - a);
    const float wcur = a[std::min(want, len - 1)], wprev = want > 0 ? a[want - 1] : 0.0f;
    if (got != want || std::memcmp(&cur, &wcur, 4) != 0 || std::memcmp(&prev, &wprev, 4) != 0) ++bad;
    return std::min(got, len - 1);
  };
  for (int64_t i = 0; i < n; ++i) {
    const int row = check(t.p_theta.data(), height, t.r_theta.data(), u1[i]);
    check(&t.p_phi[(size_t)row * width], width, &t.r_phi[(size_t)row * PT_ENV_GUIDE], u2[i]);
  }
  if (long_windows) *long_windows = longw;
  return bad;
}

int pt_get_stats(pt_ctx* c, pt_stats* out) {
  if (!c || !out) return fail(PT_E_INVALID, "pt_get_stats: NULL argument");
  int rc = settle_times(c);
  if (rc) return rc;
  *out = c->last;
  return PT_OK;
}

int pt_get_launch_times(pt_ctx* c, float* kernel_ms, float* resolve_ms, int32_t cap, int32_t* n) {
  if (!c || !n || cap < 0 || (cap > 0 && !kernel_ms)) return fail(PT_E_INVALID, "pt_get_launch_times: bad args");
  int64_t k = std::min<int64_t>({(int64_t)cap, c->n_launches, (int64_t)pt_ctx::kRing});
  *n = (int32_t)k;
  if (k == 0) return PT_OK;
  HIPCHK(hipSetDevice(c->device));
  for (int64_t i = 0; i < k; ++i) {
    hipEvent_t* tri = c->ev[(c->n_launches - k + i) % pt_ctx::kRing];
    HIPCHK(hipEventSynchronize(tri[2]));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, tri[0], tri[1]));
    kernel_ms[i] = ms;
    if (resolve_ms) {
      HIPCHK(hipEventElapsedTime(&ms, tri[1], tri[2]));
      resolve_ms[i] = ms;
    }
  }
  return PT_OK;
}

int pt_get_wave_trace(pt_ctx* c, int64_t* out, int64_t cap, int64_t* n_waves) {
  if (!c || !n_waves) return fail(PT_E_INVALID, "pt_get_wave_trace: NULL argument");
  if (!c->last.counters_valid && !c->census_valid)
    return fail(PT_E_INVALID, "pt_get_wave_trace: the last launch had no counters (or census)");
  const int64_t n = c->last.grid_blocks;
  *n_waves = n;
  if (!out) return PT_OK;
  if (cap < n * PT_WAVE_TRACE) return fail(PT_E_INVALID, "pt_get_wave_trace: buffer too small");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipMemcpy(out, c->stats.p + PT_STATS_SLOTS, (size_t)n * PT_WAVE_TRACE * sizeof(int64_t),
                   hipMemcpyDeviceToHost));
  return PT_OK;
}

}  // extern "C"
