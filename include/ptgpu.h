/* ptgpu.h — C ABI of the MI355X-native path-tracing hot path.
 *
 * This is the drop-in boundary for the reference's per-pixel radiance loop.
 * Every entry point names the reference interface it replaces:
 *
 *   pt_create / pt_destroy      CUDAPathTracer::CUDAPathTracer / ~CUDAPathTracer
 *                               (cuda_src/setup.h:90-148, setup.cu:92-115)
 *   pt_upload_scene             CUDAPathTracer::init -> loadPrimitives/loadLights/
 *                               loadBVH (setup.cu:181-201, 249-476, 689-774).  The
 *                               render tree is the library's own binned-SAH BVH over
 *                               the handed-over primitives (the nearest
 *                               hit does not depend on the tree); scene.nodes (the
 *                               reference's tree) is validated and kept for
 *                               PT_FLAG_REF_COUNTS, and rendered over when the
 *                               environment sets PT_BVH_BUILD=ref.  Primitive ids
 *                               reported anywhere stay in the caller's order.
 *   pt_upload_scene_lbvh        the same with the BVH built on the GPU: the reference's
 *                               PARALLEL_BUILD_BVH path CUDAPathTracer::buildBVH
 *                               (setup.cu:188-189, 478-686; kernel.cu:358-493) —
 *                               scene.nodes is ignored (may be NULL)
 *   pt_set_camera               CUDAPathTracer::loadCamera (setup.cu:221-247);
 *                               camera semantics of Camera::generate_ray
 *                               (src/camera.cpp:113-129)
 *   pt_set_params               CUDAPathTracer::loadParameters (setup.cu:777-811);
 *                               PathTracer::ns_aa/max_ray_depth/ns_area_light
 *                               (src/pathtracer.h:222-227)
 *   pt_render_tiles             PathTracer::raytrace_tile(tile_x,tile_y,tile_w,tile_h)
 *                               (src/pathtracer.h:181, src/pathtracer.cpp:585-611) for
 *                               one tile; whole-frame batches replace
 *                               CUDAPathTracer::startRayTracingPT + updateHostSampleBuffer
 *                               + PathTracer::updateBufferFromGPU (setup.cu:147-179,813-843)
 *   pt_tile_submit / pt_tile_finish   raytrace_tile from the reference's worker threads,
 *                               asynchronous: tiles batched into launches, each completed
 *                               (sampleBuffer + toColor) by a completion thread
 *   pt_render_tiles_device      same, output left in device memory on a caller stream
 *                               (used for the multi-GPU framebuffer reduction)
 *   pt_render_frames_device     several frames of one tile set (one seed each) in one
 *                               launch: CUDAPathTracer::startRayTracingPT called back to
 *                               back (setup.cu:147-179), without a drain between frames
 *   pt_intersect                BVHAccel::intersect(ray, isect) and BVHAccel::intersect(ray)
 *                               (src/bvh.cpp:331-362) as a batched query
 *   pt_get_stats                timers/counters (pathtracer.cpp:615-632, setup.cu:546-685)
 *   pt_last_error               replaces fprintf+exit(EXIT_FAILURE) (setup.cu:139-143, ...)
 *
 * Conventions: plain C types and host pointers only; the caller owns every host
 * input and output; the library owns device memory until pt_destroy.  Calls on
 * one pt_ctx are serialised by the caller; different contexts (one per GPU) may
 * be driven from different host threads or processes.  Every function returns
 * PT_OK (0) or a negative PT_E_* code and never exits the process.
 * Image layout: float32 RGB, row-major, index (x + y*W)*3, y = 0 is the BOTTOM
 * row (HDRImageBuffer::update_pixel, src/image.h:113-117).
 */
#ifndef PTGPU_H
#define PTGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PT_OK 0
#define PT_E_INVALID (-1)  /* bad argument / unsupported scene content */
#define PT_E_HIP (-2)      /* HIP runtime error (message in pt_last_error) */
#define PT_E_NOSCENE (-3)  /* render/intersect before pt_upload_scene/pt_set_camera */
#define PT_E_ALLOC (-4)    /* device or host allocation failed */
#define PT_E_IO (-5)       /* file could not be read/written */

/* Primitive types follow Primitive::getType(): Sphere 0, Triangle 1. */
#define PT_PRIM_SPHERE 0
#define PT_PRIM_TRIANGLE 1
/* BSDF types follow BSDF::getType(): Diffuse 0, Mirror 1, Refraction 2, Glass 3, Emission 4. */
#define PT_BSDF_DIFFUSE 0
#define PT_BSDF_MIRROR 1
#define PT_BSDF_REFRACTION 2
#define PT_BSDF_GLASS 3
#define PT_BSDF_EMISSION 4
/* Light types follow SceneLight::getType(): Directional 0, Hemisphere 1, Point 2, Area 3;
 * Environment 4 (EnvironmentLight, src/static_scene/environment_light.cpp, whose own
 * getType() says 1) — its map is pt_scene.env_*; at most one, last in the list as
 * PathTracer::set_scene pushes it (src/pathtracer.cpp:88-90). */
#define PT_LIGHT_DIRECTIONAL 0
#define PT_LIGHT_HEMISPHERE 1
#define PT_LIGHT_POINT 2
#define PT_LIGHT_AREA 3
#define PT_LIGHT_ENVIRONMENT 4

typedef struct pt_ctx pt_ctx;

/* One BSDF (src/bsdf.h).  albedo holds Diffuse::albedo, Mirror::reflectance and
 * Glass::reflectance; transmittance holds Refraction/Glass::transmittance;
 * emission holds EmissionBSDF::radiance. */
typedef struct pt_bsdf {
  int32_t type;
  float albedo[3];
  float transmittance[3];
  float emission[3];
  float ior;
  float roughness;
} pt_bsdf;

/* One light (src/static_scene/light.h).  Directional: direction = dirToLight.
 * Point: position.  Area: position, direction, dim_x, dim_y, area. */
typedef struct pt_light {
  int32_t type;
  float radiance[3];
  double position[3];
  double direction[3];
  double dim_x[3];
  double dim_y[3];
  float area;
} pt_light;

/* Camera (src/camera.h): pos, c2w(i,j) row-major, screenW/H/screenDist. */
typedef struct pt_camera {
  double pos[3];
  double c2w[9];
  double screen_w;
  double screen_h;
  double screen_dist;
} pt_camera;

/* One node of the reference BVH (src/bvh.h BVHNode), flattened: children by
 * index (-1 = NULL), primitives [start, start+range) of the BVH-ordered list. */
typedef struct pt_bvh_node {
  double bb_min[3];
  double bb_max[3];
  int64_t start;
  int64_t range;
  int64_t left;
  int64_t right;
} pt_bvh_node;

/* Flattened scene exactly as BVHAccel holds it: primitives in BVH order.
 * prim_geom: triangle p1,p2,p3 (9 doubles); sphere o.xyz, r (rest 0).
 * prim_norm: triangle vertex normals n1,n2,n3 (9 doubles); sphere ignored.
 * nodes[0] is the root. */
typedef struct pt_scene {
  int64_t n_prims;
  const int32_t* prim_type;
  const int32_t* prim_bsdf;
  const double* prim_geom;
  const double* prim_norm;
  int64_t n_nodes;
  const pt_bvh_node* nodes;
  int32_t n_bsdfs;
  const pt_bsdf* bsdfs;
  int32_t n_lights;
  const pt_light* lights;
  /* HDRImageBuffer of the environment light (NULL / 0 when there is none):
   * env_width x env_height float RGB, row 0 = +y (theta = (y+0.5)/h*pi). */
  int32_t env_width;
  int32_t env_height;
  const float* env_rgb;
} pt_scene;

/* Integrator settings (PathTracer members) and frame size. */
typedef struct pt_params {
  int32_t width;         /* 1 .. 65535 (and width * height <= 2^30) */
  int32_t height;        /* 1 .. 65535 */
  int32_t spp;           /* ns_aa */
  int32_t max_depth;     /* max_ray_depth, 0 .. 254 */
  int32_t ns_area_light; /* ns_area_light, 1 .. 255 */
  uint32_t seed;         /* counter-RNG key: (seed, pixel, sample) */
  uint32_t sample_base;  /* first sample index of this pass: samples sample_base .. sample_base+spp-1
                            are rendered and averaged (0 = the reference's single pass; progressive
                            passes / the multi-GPU sample split use disjoint ranges) */
} pt_params;

typedef struct pt_tile {
  int32_t x, y, w, h;
} pt_tile;

typedef struct pt_stats {
  int64_t pixels;       /* pixels rendered by the last call */
  int64_t samples;      /* pixels * spp */
  int64_t camera_rays;
  int64_t bounce_rays;
  int64_t shadow_rays;
  int64_t node_visits;  /* BVH2 internal-node fetches (64 B each in the reference layout) */
  int64_t tri_tests;
  int64_t sphere_tests;
  int64_t ext_hits;     /* nearest-hit rays that hit (shading-normal fetch) */
  double last_ms;       /* device time of the last render kernel (hipEvent) */
  int32_t counters_valid; /* 1 if the last call ran with PT_FLAG_STATS */
  int32_t grid_blocks;    /* persistent workgroups launched (PT_BLOCK lanes each) */
  int32_t blocks_per_cu;  /* resident workgroups per CU the occupancy query allows */
  int64_t wave_trav_steps; /* wave-level traversal steps (SIMD efficiency = node_visits / (64 * this)) */
  int64_t wave_rounds;     /* wave-level shading/refill rounds */
  int64_t culled_samples;  /* samples of pixels outside the scene's screen footprint (radiance 0, not traced) */
  int64_t queue_atomics;   /* work-queue atomics issued */
  int64_t shade_clocks;    /* shader clocks summed over waves: everything but traversal (shading, refill,
                              camera rays, loop overhead); shade_clocks + trav_clocks = the waves' summed
                              lifetimes.  All *_clocks come from the PT_FLAG_STATS build of the kernel,
                              which runs slower than the plain build (counters and clock stamps) */
  int64_t trav_clocks;     /* shader clocks summed over waves: traversal phases */
  int64_t max_wave_clocks; /* shader clocks of the slowest wave */
  int64_t wave_wall_sum;   /* wave lifetimes summed, device wall-clock ticks */
  int64_t wave_wall_max;   /* longest wave lifetime, device wall-clock ticks */
  int64_t leaf_steps;      /* of wave_trav_steps: leaf (primitive) steps */
  int64_t hitshade_clocks; /* of shade_clocks: hit records, NEE and bounces = section_clocks[0..2] */
  double resolve_ms;       /* device time of the sample-group resolve kernel */
  int32_t bvh_stack;       /* worst-case traversal stack entries of the uploaded BVH */
  int64_t bvh_nodes;       /* render-tree (BVH4) nodes uploaded */
  int64_t section_clocks[4]; /* of shade_clocks: hit record, light sampling, BSDF sampling + sample
                                completion, queue fetch (the rest of shade_clocks: camera rays and loop
                                overhead) */
  int64_t wave_span[5];    /* wall-clock ticks after the first wave started: last wave start,
                              first wave end, last wave end, first and last time a wave found
                              the work queue empty (launch ramp, queue drain and tail) */
  int32_t group_spp;       /* samples per work slot (pixel, sample group) of the last launch */
  int64_t lane_iters[4];   /* traversal lane-iterations (64 per wave iteration) spent at the other
                              step kind, finished and waiting for the shading round, retired
                              (queue drained), stepping a leaf; node steps = node_visits */
  int64_t deep_stack_steps; /* traversal lane-steps taken while the ray's stack held entries beyond the
                              PT_STACK (24) kept in LDS, i.e. in the global spill area */
  int64_t partial_bytes;   /* device bytes of the sample-group sums of the last launch: 12 B per work slot
                              of its own blocks (pixels * ceil(spp/group_spp) * 12 at most; a rank
                              rendering 1/N of a frame's tiles holds 1/N of them; two render slots
                              pipeline renders) */
  int32_t footprint[4];    /* the scene's screen footprint of the last launch, x0, y0, x1, y1 inclusive and
                              clamped to the frame: every pixel outside it has radiance 0 for every sample
                              (its camera ray misses the scene box; not traced).  The whole frame when
                              culling is off (environment light, camera not in front of the box); the
                              empty rectangle (0, 0, -1, -1) when the box is entirely off-screen. */
  int64_t slot_latency_hist[32]; /* PT_FLAG_STATS: work slots by wall-clock latency (first camera ray to the
                              group's store), bucket b = [2^(b-1), 2^b) microseconds (0: < 1 us, 31: the
                              rest) */
  int64_t node_census[8];  /* PT_FLAG_STATS: wave node steps of the traversal loop (root steps of fresh rays
                              apart); of them with every stepping lane at one node (a scalar-load
                              candidate); lanes at the first stepping lane's node; stepping lanes; steps and
                              lanes inside the top two BVH4 levels below the root (node index < 21 in the
                              breadth-first order); the same for three levels (< 85) */
  int32_t frames_per_launch; /* frames the last render launch held (pt_render_frames_device batches: up to
                                PT_MAX_FRAMES; 1 otherwise) */
  int32_t tile_zorder; /* 1: the last launch rendered its tiles in Z-order (large frames over trees above
                          PT_BANDS_TREE_MIB; PT_TILE_ZORDER=0/1 forces it) -- the same image */
} pt_stats;

#define PT_FLAG_STATS 1u /* count rays / node visits / primitive tests (slower build of the kernel) */
#define PT_FLAG_REF_COUNTS 2u /* as PT_FLAG_STATS, but traverse the reference's binary BVH so node_visits
                                 and primitive tests follow SURVEY.md §8(d)'s reference-layout cost model */

#define PT_FLAG_PACKED 4u /* pt_render_tiles_device only: hdr_out_dev holds n_tiles*32*32*3 floats and
                             tile i's pixel (x, y) goes to [(i*1024 + (y-tile.y)*32 + (x-tile.x))*3]
                             (every tile 1..32 x 1..32 and inside the frame); the multi-GPU exchange
                             gathers these packed tiles instead of whole frames */
#define PT_FLAG_PACKED16 8u /* as PT_FLAG_PACKED with 16x16 slots: n_tiles*16*16*3 floats, tile i's pixel
                               (x, y) at [(i*256 + (y-tile.y)*16 + (x-tile.x))*3], every tile 1..16 x 1..16
                               (the strong split dealing 16x16 tiles: a rank's share spread more evenly) */

int pt_create(int device, pt_ctx** out);
int pt_destroy(pt_ctx* ctx);
int pt_upload_scene(pt_ctx* ctx, const pt_scene* scene);
/* Uploads the scene and builds a linear BVH on the device (Morton codes,
 * radix sort, Karras tree, bottom-up boxes, leaves of <= 4 primitives, then
 * the 4-wide layout).  Primitive indices reported by pt_intersect stay those
 * of the uploaded arrays. */
int pt_upload_scene_lbvh(pt_ctx* ctx, const pt_scene* scene);
int pt_set_camera(pt_ctx* ctx, const pt_camera* cam);
int pt_set_params(pt_ctx* ctx, const pt_params* params);
/* Renders the listed tiles into a host framebuffer of width*height*3 floats;
 * only pixels inside the tiles are written.  flags: PT_FLAG_* */
int pt_render_tiles(pt_ctx* ctx, const pt_tile* tiles, int32_t n_tiles, float* hdr_out_host,
                    uint32_t flags);
/* Same, into a device framebuffer (width*height*3 floats) on `stream`
 * (hipStream_t, NULL = the context's stream).  Returns after the kernel is
 * queued, without waiting for it (a PT_FLAG_STATS / PT_FLAG_REF_COUNTS call
 * waits, to read its counters); synchronise on the stream before reading.
 * The framebuffer is written in `stream` order: after the work queued on
 * `stream` before the call, before the work queued after it (the kernels
 * themselves run on the context's render streams).
 * Replaces CUDAPathTracer::startRayTracingPT (cuda_src/setup.cu:147-179)
 * minus its host copy-back. */
int pt_render_tiles_device(pt_ctx* ctx, const pt_tile* tiles, int32_t n_tiles, float* hdr_out_dev,
                           void* stream, uint32_t flags);
/* A frame batch: n_frames (1..PT_MAX_FRAMES = 8) renders of the same tiles, frame
 * f with pt_params.seed replaced by seeds[f], into hdr_outs_dev[f] (each as
 * pt_render_tiles_device's hdr_out_dev, PT_FLAG_PACKED allowed; counters are
 * not: PT_FLAG_STATS / PT_FLAG_REF_COUNTS return PT_E_INVALID).  Every image
 * is bit-identical to its own pt_render_tiles_device call with that seed;
 * the frames share ONE persistent launch, so a small frame's drain (a rank's
 * share of a split frame) is filled with the next frame's work.  Stream
 * semantics as pt_render_tiles_device. */
#define PT_MAX_FRAMES 8
int pt_render_frames_device(pt_ctx* ctx, const pt_tile* tiles, int32_t n_tiles, int32_t n_frames,
                            const uint32_t* seeds, float* const* hdr_outs_dev, void* stream, uint32_t flags);
/* Asynchronous one-tile seam: PathTracer::raytrace_tile(tile_x, tile_y, tile_w, tile_h)
 * (src/pathtracer.cpp:585-611) as the reference's worker threads call it
 * (worker_thread, pathtracer.cpp:613-621), without one launch and one host
 * synchronisation per tile.  pt_tile_submit queues the tile and returns; queued
 * tiles render as ONE launch once PT_TILE_BATCH (default 256) are queued, or at
 * pt_tile_finish.  When a tile's launch completes, its pixels are written into
 * hdr_out_host (the width*height*3 sampleBuffer) and, if rgba_out_host is not
 * NULL, toColor'd into it (the width*height frameBuffer, as pt_to_color), by the
 * context's completion thread, which waits on each launch's event off the
 * render stream (so completing one batch overlaps the next batch's render) --
 * exactly what raytrace_tile leaves behind.  At most 8 launched batches await
 * completion; a submit beyond that waits for one.  The caller keeps
 * both buffers alive and does not write the tile's pixels until pt_tile_finish
 * returns.  pt_tile_finish renders what is still queued and waits for every
 * submitted tile.  Tiles render with the scene/camera/params of submission
 * (the setters and the synchronous renders first launch what is queued).  The
 * pixels equal those of a whole-frame pt_render_tiles bit for bit.  A failed
 * launch or completion is returned by the call that hit it (a launch) and
 * ALSO by the next pt_tile_finish: its tiles were not rendered.  Whatever it
 * returns, pt_tile_finish returns only after every launched batch has been
 * completed, so the caller's buffers stay in use until pt_tile_finish returns
 * and are free afterwards, on success or error. */
int pt_tile_submit(pt_ctx* ctx, const pt_tile* tile, float* hdr_out_host, uint32_t* rgba_out_host);
int pt_tile_finish(pt_ctx* ctx);
/* Batched BVHAccel::intersect.  Rays: origin o[3n], direction d[3n] (normalised),
 * max_t[n] for the any-hit query.  Outputs (each nullable): nearest hit flag,
 * t, primitive index (the caller's BVH order, whatever tree renders), and the any-hit
 * flag within (0, max_t). */
int pt_intersect(pt_ctx* ctx, int64_t n, const double* o, const double* d, const double* max_t,
                 int32_t* hit, float* t, int32_t* prim, int32_t* any_hit);
/* Statistics of the last render (waits for its kernel-time events). */
int pt_get_stats(pt_ctx* ctx, pt_stats* out);
/* Kernel and resolve times in ms of the last min(cap, launches, 256) renders,
 * oldest first (waits for them); *n = how many were written.  resolve_ms may
 * be NULL.  No reference counterpart (its timers are host wall-clock,
 * application.cpp:776-780): the HIP-event view of the same launches. */
int pt_get_launch_times(pt_ctx* ctx, float* kernel_ms, float* resolve_ms, int32_t cap, int32_t* n);
/* Diagnostics (no reference counterpart): after a PT_FLAG_STATS launch, one
 * record of 11 int64 per wave -- device wall-clock start, first time the wave
 * found the work queue empty (~0 if never), end, (XCC id << 32 | HW_ID), the
 * camera samples it started, the sum and maximum of its work slots'
 * latencies (claim to partial-sum store, wall-clock ticks), the most
 * traversal iterations one ray stepped in (<< 32) | sat out, the most
 * traversal phases one ray spanned, and the traversal iterations and shading
 * rounds it ran after it saw the queue drained.  out == NULL: only *n_waves
 * is set. */
int pt_get_wave_trace(pt_ctx* ctx, int64_t* out, int64_t cap, int64_t* n_waves);
const char* pt_last_error(void);

/* Output row, host side (no device needed):
 * HDRImageBuffer::toColor(target, x0, y0, x1, y1) (src/image.h:174-189) of the
 * HDR buffer `hdr` (width*height*3 float, the sampleBuffer layout) into the
 * RGBA8 `frame` (width*height uint32, ImageBuffer::data: r | g<<8 | b<<16 |
 * a<<24, image.h:49-58), with the reference's float arithmetic (powf; NaN ->
 * 255).  Pixels outside [x0,x1) x [y0,y1) are left untouched. */
int pt_to_color(const float* hdr, int32_t width, int32_t height, int32_t x0, int32_t y0, int32_t x1, int32_t y1,
                uint32_t* frame);
/* Diagnostics for pt_to_color's tabulated codes: the number of float bit patterns in
 * [lo_bits, hi_bits) whose tabulated 8-bit code differs from the direct evaluation
 * code8(powf(s * exposure, 1 / 2.2)) (0 = the table is exact there). */
int64_t pt_to_color_check(uint32_t lo_bits, uint32_t hi_bits);
/* Diagnostics for the environment light's inverse-CDF sampling (host only): builds
 * EnvironmentLight's tables (src/static_scene/environment_light.cpp:6-48) for the
 * width x height float RGB map and replays the kernel's guide-record search
 * (pt_device.h record_lower_bound) for n query pairs (u1[i], u2[i]) in [0, 1)
 * against std::lower_bound, as importanceSampling's two searches
 * (environment_light.cpp:69-115): returns how many searches disagreed in the index
 * or the interpolation pair (0 = exact), or a negative PT_E_*; *long_windows (nullable)
 * receives how many searches took the window-halving path. */
int64_t pt_env_search_check(const float* rgb, int32_t width, int32_t height, int64_t n, const float* u1,
                            const float* u2, int64_t* long_windows);

#ifdef __cplusplus
}
#endif

#endif /* PTGPU_H */
