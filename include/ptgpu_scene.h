/* ptgpu_scene.h — native host scene pipeline of the HIP path (C ABI).
 *
 * For callers that do not own a CMU462 PathTracer: restates the reference's
 * host side that produces the flattened scene pt_upload_scene consumes.
 *
 *   pt_host_scene_load   Collada::ColladaParser::load (src/collada/collada.cpp:131-936)
 *                        + Application::load / init_* (src/application.cpp:223-365)
 *                        + DynamicScene -> StaticScene (src/dynamic_scene/{mesh,sphere,scene}.cpp,
 *                          src/static_scene/object.cpp:16-80)
 *                        + HalfedgeMesh::build / Vertex::computeNormal
 *                          (src/halfEdgeMesh.cpp:29-397, src/halfEdgeMesh.h:492-515)
 *                        + PathTracer::build_accel / BVHAccel::BVHAccel / buildBVH
 *                          (src/pathtracer.cpp:224-248, src/bvh.cpp:21-202; with the
 *                          bucket-index clamp of SURVEY.md §8(a) quirk 1)
 *                        + Application::loadCamera for .info files
 *                          (src/application.cpp:823-853)
 *   pt_host_scene_view   borrowed pt_scene / pt_camera views of the result
 *   pt_host_scene_dump   PTDUMP file (the oracle's scene interchange format)
 *   pt_host_scene_free   release
 *   pt_host_load_exr     load_exr (src/main.cpp:30-67) over tinyexr: an OpenEXR
 *                        environment map as float RGB (scanline; NONE/ZIPS/ZIP;
 *                        HALF/FLOAT), channels 2,1,0 of the name-sorted list as R,G,B
 *
 * The result is bit-identical to what the reference's own host code builds
 * (primitive order, vertex order, area-weighted normals, BVH topology and
 * boxes, lights, BSDFs, camera); tests/test_scene_loader.py pins it against
 * dumps written by the reference (oracle/_ref/ref_driver --mode dump).
 */
#ifndef PTGPU_SCENE_H
#define PTGPU_SCENE_H

#include <stdint.h>

#include "ptgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pt_host_scene pt_host_scene;

/* Loads a COLLADA .dae, builds the reference BVH and places the default camera
 * for a width x height frame.  cam_info (nullable) is a .info camera file. */
int pt_host_scene_load(const char* dae_path, int32_t width, int32_t height, const char* cam_info,
                       pt_host_scene** out);
/* Borrowed views, valid until pt_host_scene_free. Either pointer may be NULL. */
int pt_host_scene_view(const pt_host_scene* hs, pt_scene* scene, pt_camera* cam);
/* Adds the EnvironmentLight of an OpenEXR lat-long map (main.cpp -e +
 * PathTracer::set_scene: appended after the scene's lights). */
int pt_host_scene_set_envmap(pt_host_scene* hs, const char* exr_path);
/* Writes the flattened scene as a PTDUMP file. */
int pt_host_scene_dump(const pt_host_scene* hs, const char* path);
void pt_host_scene_free(pt_host_scene* hs);

/* The render tree pt_upload_scene traverses: this library's own
 * binned-SAH binary BVH over scene's primitives, in pt_bvh_node form (nodes[0] the
 * root, children by index, leaves of <= 4 primitives as [start, start+range) of the
 * permuted order).  perm[i] = the scene index of the i-th primitive in that order.
 * nodes must hold 2*n_prims-1 entries, perm n_prims; *n_nodes receives the count.
 * Deterministic: independent of the number of host threads used (PT_BUILD_THREADS). */
int pt_host_build_render_tree(const pt_scene* scene, pt_bvh_node* nodes, int64_t* n_nodes, int64_t* perm);

/* Reads an OpenEXR file into a malloc'd float RGB array (width*height*3, row 0
 * = first scanline = +y for lat-long maps); free it with pt_host_free. */
int pt_host_load_exr(const char* path, int32_t* width, int32_t* height, float** rgb);
void pt_host_free(void* p);

#ifdef __cplusplus
}
#endif

#endif /* PTGPU_SCENE_H */
