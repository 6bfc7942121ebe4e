// capture_abi.cpp — TEST DOUBLE of the include/ptgpu.h ABI for the
// INTEGRATION.md adapter link test (tests/test_integration_doc.py).  It
// implements the entry points GpuPathTracer calls without a GPU: every
// pt_scene / pt_camera the adapter hands over is written, field for field, to
// the PTDUMP file named by $PT_CAPTURE_OUT under the record names
// oracle/_ref/ref_driver --mode dump uses; pt_set_params and pt_render_tiles
// calls are logged ("params": 7 ints per call, "tiles": 4 ints + the seed in
// force, per call; pt_tile_submit calls the same) and leave the output buffer
// untouched; "finishes" logs the tiles submitted at each pt_tile_finish.
#include <cstdlib>
#include <vector>

#include "ptdump.h"
#include "ptgpu.h"

struct pt_ctx {
  std::vector<double> cam;
  std::vector<int32_t> ptype, pbsdf, btype, ltype, params, tiles, finishes;
  std::vector<double> pgeom, pnorm, nbb, lgeom;
  std::vector<int64_t> ninfo, env_shape;
  std::vector<float> bpar, lrad, larea, env;
  pt_params cur{};
  bool have_params = false;
};

static void flush(pt_ctx* c) {
  const char* out = std::getenv("PT_CAPTURE_OUT");
  if (!out) return;
  ptdump::Writer w(out);
  w.f8("cam", c->cam);
  w.i4("bsdf_type", c->btype);
  w.f4("bsdf_params", c->bpar);
  w.i4("light_type", c->ltype);
  w.f4("light_rad", c->lrad);
  w.f8("light_geom", c->lgeom);
  w.f4("light_area", c->larea);
  if (!c->env_shape.empty()) {
    w.i8("env_shape", c->env_shape);
    w.f4("env_rgb", c->env);
  }
  w.i4("prim_type", c->ptype);
  w.i4("prim_bsdf", c->pbsdf);
  w.f8("prim_geom", c->pgeom);
  w.f8("prim_norm", c->pnorm);
  w.f8("node_bb", c->nbb);
  w.i8("node_info", c->ninfo);
  w.i4("params", c->params);
  w.i4("tiles", c->tiles);
  w.i4("finishes", c->finishes);
}

extern "C" {

int pt_create(int, pt_ctx** out) {
  *out = new pt_ctx();
  return PT_OK;
}

int pt_destroy(pt_ctx* c) {
  flush(c);
  delete c;
  return PT_OK;
}

int pt_upload_scene(pt_ctx* c, const pt_scene* s) {
  c->ptype.assign(s->prim_type, s->prim_type + s->n_prims);
  c->pbsdf.assign(s->prim_bsdf, s->prim_bsdf + s->n_prims);
  c->pgeom.assign(s->prim_geom, s->prim_geom + 9 * s->n_prims);
  c->pnorm.assign(s->prim_norm, s->prim_norm + 9 * s->n_prims);
  for (int64_t i = 0; i < s->n_nodes; ++i) {
    const pt_bvh_node& n = s->nodes[i];
    for (int k = 0; k < 3; ++k) c->nbb.push_back(n.bb_min[k]);
    for (int k = 0; k < 3; ++k) c->nbb.push_back(n.bb_max[k]);
    c->ninfo.insert(c->ninfo.end(), {n.start, n.range, n.left, n.right});
  }
  for (int32_t i = 0; i < s->n_bsdfs; ++i) {
    const pt_bsdf& b = s->bsdfs[i];
    c->btype.push_back(b.type);
    float p[12] = {b.albedo[0], b.albedo[1], b.albedo[2], b.transmittance[0], b.transmittance[1],
                   b.transmittance[2], b.emission[0], b.emission[1], b.emission[2], b.ior, b.roughness, 0.0f};
    c->bpar.insert(c->bpar.end(), p, p + 12);
  }
  for (int32_t i = 0; i < s->n_lights; ++i) {
    const pt_light& l = s->lights[i];
    c->ltype.push_back(l.type);
    c->lrad.insert(c->lrad.end(), l.radiance, l.radiance + 3);
    const double* g[4] = {l.position, l.direction, l.dim_x, l.dim_y};
    for (int k = 0; k < 4; ++k) c->lgeom.insert(c->lgeom.end(), g[k], g[k] + 3);
    c->larea.push_back(l.area);
  }
  if (s->env_rgb) {
    c->env_shape = {s->env_height, s->env_width};
    c->env.assign(s->env_rgb, s->env_rgb + 3 * (size_t)s->env_width * s->env_height);
  }
  return PT_OK;
}

int pt_upload_scene_lbvh(pt_ctx* c, const pt_scene* s) { return pt_upload_scene(c, s); }

int pt_set_camera(pt_ctx* c, const pt_camera* cam) {
  c->cam.assign(cam->pos, cam->pos + 3);
  c->cam.insert(c->cam.end(), cam->c2w, cam->c2w + 9);
  c->cam.insert(c->cam.end(), {cam->screen_w, cam->screen_h, cam->screen_dist});
  return PT_OK;
}

int pt_set_params(pt_ctx* c, const pt_params* p) {
  c->cur = *p;
  c->have_params = true;
  c->params.insert(c->params.end(), {p->width, p->height, p->spp, p->max_depth, p->ns_area_light,
                                     (int32_t)p->seed, (int32_t)p->sample_base});
  return PT_OK;
}

int pt_render_tiles(pt_ctx* c, const pt_tile* tiles, int32_t n, float*, uint32_t) {
  if (!c->have_params) return PT_E_NOSCENE;
  for (int32_t i = 0; i < n; ++i)
    c->tiles.insert(c->tiles.end(), {tiles[i].x, tiles[i].y, tiles[i].w, tiles[i].h, (int32_t)c->cur.seed});
  return PT_OK;
}

int pt_tile_submit(pt_ctx* c, const pt_tile* t, float* hdr, uint32_t*) {
  if (!c->have_params || !hdr) return PT_E_NOSCENE;
  c->tiles.insert(c->tiles.end(), {t->x, t->y, t->w, t->h, (int32_t)c->cur.seed});
  return PT_OK;
}

int pt_tile_finish(pt_ctx* c) {
  c->finishes.push_back((int32_t)(c->tiles.size() / 5));  // tiles submitted when the frame was finished
  return PT_OK;
}

const char* pt_last_error(void) { return "capture ABI"; }

}  // extern "C"
