// ref_driver.cpp — ORACLE TEST INFRASTRUCTURE (never shipped, never measured as
// the product).  A headless harness around the reference's OWN CPU path-tracer
// sources (/root/reference/src, compiled unmodified except the bucket-index
// clamp in bvh.cpp:47, see oracle/ref/Makefile).  It replaces only the GUI
// driver (src/main.cpp + src/application.cpp, which need GLFW/freetype/GLU that
// this image lacks) with a restatement of the few lines of scene set-up they
// perform:
//   * scene load: Collada::ColladaParser::load        (src/main.cpp:132-136)
//   * Application::load object/light/camera creation  (src/application.cpp:223-299)
//   * Application::set_up_pathtracer                  (src/application.cpp:624-633)
//   * Application::loadCamera (-f cam.info)           (src/application.cpp:823-853)
//   * srand + start_raytracing + wait for DONE        (src/main.cpp:75,170-181)
// Modes:
//   render : writes the HDR sampleBuffer (float32 W*H*3, y=0 bottom) to a PTDUMP
//   tiles  : times PathTracer::raytrace_tile (pathtracer.cpp:585-611) on every
//            --tile-stride-th 32x32 tile of the FIFO from --tile-begin, on this
//            one thread (the -t 1 worker's work, glibc rand() as shipped), or
//            with -t T on T threads popping those tiles from one shared queue
//            as the reference's workers do (its published -t 8 setting) — the
//            CPU baselines of bench.py on a bounded sample of a frame
//   dump   : writes the flattened scene the GPU seam would receive (PTDUMP)
//   rays   : answers BVHAccel::intersect nearest/any-hit queries (KATs)
//   rng    : prints the first rand() draws and the sampler draw order
//   exr    : decodes --envmap with the reference's tinyexr + load_exr (main.cpp:30-67)
//            and writes the HDRImageBuffer (float32 w*h*3) to a PTDUMP
//   tocolor: HDRImageBuffer::toColor (image.h:174-189) of the PTDUMP "hdr" of --in
//            into the RGBA8 frameBuffer, plus the vertically flipped copy
//            PathTracer::save_image hands lodepng (pathtracer.cpp:649-674)
//   exrw   : writes the PTDUMP "rgb" (w, h) of --in as a ZIP OpenEXR with the
//            reference's tinyexr (SaveMultiChannelEXRToFile), channels B,G,R,
//            pixel type --half 0/1 (fixtures for the native EXR loader)
// --envmap <file.exr> adds the EnvironmentLight exactly as main.cpp -e does:
// PathTracer(..., envmap) pushes it after the scene's lights (pathtracer.cpp:42-46,88-90).
// the reference's tinyexr, implemented in this TU as src/main.cpp:4 does
// (first, so no earlier include of the header swallows the implementation)
#define TINYEXR_IMPLEMENTATION
#include "tinyexr.h"
#include "pathtracer.h"
#include "bsdf.h"
#include "camera.h"
#include "collada/collada.h"
#include "dynamic_scene/ambient_light.h"
#include "dynamic_scene/area_light.h"
#include "dynamic_scene/directional_light.h"
#include "dynamic_scene/point_light.h"
#include "dynamic_scene/mesh.h"
#include "dynamic_scene/sphere.h"
#include "dynamic_scene/scene.h"
#include "static_scene/light.h"
#include "static_scene/sphere.h"
#include "static_scene/triangle.h"

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "ptdump.h"
#include "static_scene/environment_light.h"

using namespace CMU462;
using std::string;
using std::vector;

struct Opts {
  string scene, mode = "render", out, cam, rays_in, envmap, in;
  int half = 0;
  size_t w = 64, h = 64, spp = 1, depth = 4, lights = 1, threads = 1;
  size_t tile_begin = 0, tile_stride = 1;
  unsigned seed = 1;
};

static HDRImageBuffer* g_envmap = nullptr;  // --envmap, owned by the EnvironmentLight

static void die(const char* m) {
  std::fprintf(stderr, "ref_driver: %s\n", m);
  std::exit(2);
}

// Restatement of Application::load (application.cpp:223-299) minus GL state.
static void build_scene(const Opts& o, Camera& camera, DynamicScene::Scene*& dscene) {
  Collada::SceneInfo* sceneInfo = new Collada::SceneInfo();
  if (Collada::ColladaParser::load(o.scene.c_str(), sceneInfo) < 0) die("cannot load scene");
  vector<DynamicScene::SceneLight*> lights;
  vector<DynamicScene::SceneObject*> objects;
  Vector3D c_pos, c_dir;
  for (Collada::Node& node : sceneInfo->nodes) {
    Collada::Instance* instance = node.instance;
    const Matrix4x4& transform = node.transform;
    switch (instance->type) {
      case Collada::Instance::CAMERA: {
        Collada::CameraInfo* c = static_cast<Collada::CameraInfo*>(instance);
        c_pos = (transform * Vector4D(c_pos, 1)).to3D();
        c_dir = (transform * Vector4D(c->view_dir, 1)).to3D().unit();
        camera.configure(*c, o.w, o.h);
        break;
      }
      case Collada::Instance::LIGHT: {
        Collada::LightInfo& li = static_cast<Collada::LightInfo&>(*instance);
        DynamicScene::SceneLight* l = nullptr;
        switch (li.light_type) {
          case Collada::LightType::AMBIENT: l = new DynamicScene::AmbientLight(li); break;
          case Collada::LightType::DIRECTIONAL: l = new DynamicScene::DirectionalLight(li, transform); break;
          case Collada::LightType::AREA: l = new DynamicScene::AreaLight(li, transform); break;
          case Collada::LightType::POINT: l = new DynamicScene::PointLight(li, transform); break;
          default: break;
        }
        lights.push_back(l);
        break;
      }
      case Collada::Instance::SPHERE: {
        Collada::SphereInfo& s = static_cast<Collada::SphereInfo&>(*instance);
        const Vector3D& position = (transform * Vector4D(0, 0, 0, 1)).projectTo3D();
        double scale = (transform * Vector4D(1, 0, 0, 0)).to3D().norm();
        objects.push_back(new DynamicScene::Sphere(s, position, scale));
        break;
      }
      case Collada::Instance::POLYMESH:
        objects.push_back(new DynamicScene::Mesh(static_cast<Collada::PolymeshInfo&>(*instance), transform));
        break;
      default:
        break;
    }
  }
  dscene = new DynamicScene::Scene(objects, lights);
  const BBox& bbox = dscene->get_bbox();
  if (!bbox.empty()) {
    Vector3D target = bbox.centroid();
    double canonical_view_distance = bbox.extent.norm() / 2 * 1.5;
    double view_distance = canonical_view_distance * 2;
    camera.place(target, acos(c_dir.y), atan2(c_dir.x, c_dir.z), view_distance,
                 canonical_view_distance / 10.0, canonical_view_distance * 20.0);
  }
}

// Restatement of load_exr (src/main.cpp:30-67): channels taken by index
// 2,1,0 of the file's (name-sorted) channel list as R,G,B.
static HDRImageBuffer* load_exr(const char* file_path) {
  const char* err;
  EXRImage exr;
  InitEXRImage(&exr);
  int ret = ParseMultiChannelEXRHeaderFromFile(&exr, file_path, &err);
  if (ret != 0) die("cannot parse EXR header");
  for (int i = 0; i < exr.num_channels; i++)
    if (exr.pixel_types[i] == TINYEXR_PIXELTYPE_HALF) exr.requested_pixel_types[i] = TINYEXR_PIXELTYPE_FLOAT;
  ret = LoadMultiChannelEXRFromFile(&exr, file_path, &err);
  if (ret != 0) die("cannot load EXR");
  HDRImageBuffer* envmap = new HDRImageBuffer();
  envmap->resize(exr.width, exr.height);
  float* channel_r = (float*)exr.images[2];
  float* channel_g = (float*)exr.images[1];
  float* channel_b = (float*)exr.images[0];
  for (size_t i = 0; i < (size_t)exr.width * exr.height; i++)
    envmap->data[i] = Spectrum(channel_r[i], channel_g[i], channel_b[i]);
  return envmap;
}

// tocolor: --in PTDUMP {hdr f4 (h*w*3, row 0 = y 0), shape i8 (h, w, 3)} ->
// --out {frame u4 (h*w, ImageBuffer::data), png_rows u4 (save_image's rows)}
static int tocolor_mode(const Opts& o) {
  std::vector<ptdump::Record> R;
  if (!ptdump::read_all(o.in.c_str(), R)) die("cannot read --in");
  vector<float> hdr;
  vector<int64_t> shape;
  if (!ptdump::get(R, "hdr", hdr) || !ptdump::get(R, "shape", shape) || shape.size() != 3) die("bad --in");
  const size_t h = (size_t)shape[0], w = (size_t)shape[1];
  HDRImageBuffer sb;
  sb.resize(w, h);
  for (size_t i = 0; i < w * h; ++i) sb.data[i] = Spectrum(hdr[3 * i], hdr[3 * i + 1], hdr[3 * i + 2]);
  ImageBuffer fb;
  fb.resize(w, h);
  sb.toColor(fb, 0, 0, w, h);
  vector<uint32_t> rows(w * h);  // save_image (pathtracer.cpp:662-667)
  for (size_t i = 0; i < h; ++i) std::memcpy(&rows[i * w], &fb.data[(h - i - 1) * w], 4 * w);
  ptdump::Writer wr(o.out.c_str());
  wr.raw("frame", "u4", fb.data.data(), (int64_t)(w * h), 4);
  wr.raw("png_rows", "u4", rows.data(), (int64_t)(w * h), 4);
  return 0;
}

static int exr_modes(const Opts& o) {
  if (o.mode == "exr") {
    HDRImageBuffer* m = load_exr(o.envmap.c_str());
    ptdump::Writer w(o.out.c_str());
    vector<float> rgb(m->w * m->h * 3);
    for (size_t i = 0; i < m->w * m->h; ++i) {
      rgb[3 * i] = m->data[i].r;
      rgb[3 * i + 1] = m->data[i].g;
      rgb[3 * i + 2] = m->data[i].b;
    }
    w.f4("rgb", rgb);
    w.i8("shape", {(int64_t)m->h, (int64_t)m->w, 3});
    return 0;
  }
  // exrw: PTDUMP {rgb f4 (h*w*3), shape i8 (h, w, 3)} -> ZIP EXR (B, G, R)
  std::vector<ptdump::Record> R;
  if (!ptdump::read_all(o.in.c_str(), R)) die("cannot read --in");
  vector<float> rgb;
  vector<int64_t> shape;
  if (!ptdump::get(R, "rgb", rgb) || !ptdump::get(R, "shape", shape) || shape.size() != 3) die("bad --in");
  int h = (int)shape[0], wd = (int)shape[1];
  vector<float> ch[3];
  vector<uint16_t> hch[3];
  const char* names[3] = {"B", "G", "R"};
  for (int c = 0; c < 3; ++c) {
    ch[c].resize((size_t)wd * h);
    for (size_t i = 0; i < (size_t)wd * h; ++i) ch[c][i] = rgb[3 * i + (2 - c)];
  }
  EXRImage img;
  InitEXRImage(&img);
  img.num_channels = 3;
  img.channel_names = names;
  unsigned char* ptrs[3];
  int ptype[3], rtype[3];
  for (int c = 0; c < 3; ++c) {
    ptype[c] = o.half ? TINYEXR_PIXELTYPE_HALF : TINYEXR_PIXELTYPE_FLOAT;
    rtype[c] = ptype[c];
    ptrs[c] = reinterpret_cast<unsigned char*>(ch[c].data());  // float input; converted on save
  }
  img.images = ptrs;
  img.pixel_types = ptype;
  img.requested_pixel_types = rtype;
  img.width = wd;
  img.height = h;
  if (o.half) {  // tinyexr saves HALF channels from float input data
    for (int c = 0; c < 3; ++c) ptype[c] = TINYEXR_PIXELTYPE_FLOAT;
  }
  const char* err = nullptr;
  if (SaveMultiChannelEXRToFile(&img, o.out.c_str(), &err) != 0) die(err ? err : "cannot write EXR");
  return 0;
}

// Restatement of Application::loadCamera (application.cpp:823-853).
static void load_camera_file(const string& fn, Camera& cam) {
  FILE* f = std::fopen(fn.c_str(), "r");
  if (!f) die("cannot open camera file");
  int n = 0;
  n += fscanf(f, "%lf %lf %lf", &cam.pos[0], &cam.pos[1], &cam.pos[2]);
  n += fscanf(f, "%lf %lf %lf", &cam.targetPos[0], &cam.targetPos[1], &cam.targetPos[2]);
  n += fscanf(f, "%lf", &cam.phi);
  n += fscanf(f, "%lf", &cam.theta);
  n += fscanf(f, "%lf", &cam.minR);
  n += fscanf(f, "%lf", &cam.maxR);
  n += fscanf(f, "%lf %lf %lf %lf %lf %lf %lf %lf %lf", &cam.c2w(0, 0), &cam.c2w(0, 1), &cam.c2w(0, 2),
              &cam.c2w(1, 0), &cam.c2w(1, 1), &cam.c2w(1, 2), &cam.c2w(2, 0), &cam.c2w(2, 1),
              &cam.c2w(2, 2));
  std::fclose(f);
  if (n != 19) die("bad camera file");
}

// main.cpp + Application::load + set_up_pathtracer: the PathTracer every mode uses.
static PathTracer* setup_pathtracer(const Opts& o) {
  Camera* camera = new Camera();
  DynamicScene::Scene* dscene = nullptr;
  build_scene(o, *camera, dscene);
  g_envmap = o.envmap.empty() ? nullptr : load_exr(o.envmap.c_str());
  PathTracer* pt = new PathTracer(o.spp, o.depth, o.lights, 1, 1, 1, o.threads, g_envmap);
  pt->useCPU = true;
  // set_up_pathtracer (application.cpp:624-633)
  pt->set_camera(camera);
  pt->set_scene(dscene->get_static_scene());
  pt->set_frame_size(o.w, o.h);
  if (!o.cam.empty()) load_camera_file(o.cam, *camera);
  return pt;
}

// The same set-up for the INTEGRATION.md adapter link test (tests/adapter/,
// built with -DREF_DRIVER_NO_MAIN): the PathTracer the reference's GPU seam
// would be handed, and the -e environment map (or nullptr).
PathTracer* ref_setup_pathtracer(const char* scene, size_t w, size_t h, size_t spp, size_t depth, size_t lights,
                                 const char* cam, const char* envmap, HDRImageBuffer** env_out) {
  Opts o;
  o.scene = scene;
  o.w = w;
  o.h = h;
  o.spp = spp;
  o.depth = depth;
  o.lights = lights;
  if (cam) o.cam = cam;
  if (envmap) o.envmap = envmap;
  PathTracer* pt = setup_pathtracer(o);
  if (env_out) *env_out = g_envmap;
  return pt;
}

static void dump_scene(const Opts& o, PathTracer& pt) {
  ptdump::Writer w(o.out.c_str());
  if (!w.ok()) die("cannot write dump");
  const Camera& c = *pt.camera;
  vector<double> cam = {c.pos.x, c.pos.y, c.pos.z};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) cam.push_back(c.c2w(i, j));
  cam.push_back((double)c.screenW);
  cam.push_back((double)c.screenH);
  cam.push_back(c.screenDist);
  cam.push_back(c.hFov);
  cam.push_back(c.vFov);
  w.f8("cam", cam);

  // original (collection) order: pathtracer.cpp:230-234
  std::map<const StaticScene::Primitive*, int> orig;
  for (size_t i = 0; i < pt.primitives.size(); ++i) orig[pt.primitives[i]] = (int)i;
  // BSDF table: first appearance in collection order
  std::map<const BSDF*, int> bidx;
  vector<const BSDF*> blist;
  for (StaticScene::Primitive* p : pt.primitives) {
    const BSDF* b = p->get_bsdf();
    if (!bidx.count(b)) {
      bidx[b] = (int)blist.size();
      blist.push_back(b);
    }
  }
  vector<int32_t> btype;
  vector<float> bpar;
  for (const BSDF* cb : blist) {
    BSDF* b = const_cast<BSDF*>(cb);
    float p[12] = {0};
    int t = b->getType();
    if (t == 0) { Spectrum a = static_cast<DiffuseBSDF*>(b)->albedo; p[0] = a.r; p[1] = a.g; p[2] = a.b; }
    if (t == 1) { Spectrum a = static_cast<MirrorBSDF*>(b)->reflectance; p[0] = a.r; p[1] = a.g; p[2] = a.b; }
    if (t == 2) {
      RefractionBSDF* r = static_cast<RefractionBSDF*>(b);
      p[3] = r->transmittance.r; p[4] = r->transmittance.g; p[5] = r->transmittance.b;
      p[9] = r->ior; p[10] = r->roughness;
    }
    if (t == 3) {
      GlassBSDF* g = static_cast<GlassBSDF*>(b);
      p[0] = g->reflectance.r; p[1] = g->reflectance.g; p[2] = g->reflectance.b;
      p[3] = g->transmittance.r; p[4] = g->transmittance.g; p[5] = g->transmittance.b;
      p[9] = g->ior; p[10] = g->roughness;
    }
    if (t == 4) { Spectrum e = b->get_emission(); p[6] = e.r; p[7] = e.g; p[8] = e.b; }
    btype.push_back(t);
    bpar.insert(bpar.end(), p, p + 12);
  }
  w.i4("bsdf_type", btype);
  w.f4("bsdf_params", bpar);

  vector<int32_t> ltype;
  vector<float> lrad, larea;
  vector<double> lgeom;
  const StaticScene::EnvironmentLight* env = nullptr;
  for (StaticScene::SceneLight* l : pt.scene->lights) {
    int t = l->getType();
    if (auto* e = dynamic_cast<StaticScene::EnvironmentLight*>(l)) {  // getType() says 1
      env = e;
      t = 4;
    }
    double g[12] = {0};
    Spectrum rad;
    float area = 0;
    if (t == 0) {
      auto* d = static_cast<StaticScene::DirectionalLight*>(l);
      rad = d->radiance; g[3] = d->dirToLight.x; g[4] = d->dirToLight.y; g[5] = d->dirToLight.z;
    } else if (t == 1) {
      rad = static_cast<StaticScene::InfiniteHemisphereLight*>(l)->radiance;
    } else if (t == 4) {
      // the map travels in env_rgb below
    } else if (t == 2) {
      auto* d = static_cast<StaticScene::PointLight*>(l);
      rad = d->radiance; g[0] = d->position.x; g[1] = d->position.y; g[2] = d->position.z;
    } else if (t == 3) {
      auto* a = static_cast<StaticScene::AreaLight*>(l);
      rad = a->radiance;
      const Vector3D* v[4] = {&a->position, &a->direction, &a->dim_x, &a->dim_y};
      for (int k = 0; k < 4; ++k) { g[3 * k] = v[k]->x; g[3 * k + 1] = v[k]->y; g[3 * k + 2] = v[k]->z; }
      area = a->area;
    }
    ltype.push_back(t);
    lrad.push_back(rad.r); lrad.push_back(rad.g); lrad.push_back(rad.b);
    lgeom.insert(lgeom.end(), g, g + 12);
    larea.push_back(area);
  }
  w.i4("light_type", ltype);
  w.f4("light_rad", lrad);
  w.f8("light_geom", lgeom);
  w.f4("light_area", larea);
  if (env) {
    const HDRImageBuffer* m = g_envmap;  // the map handed to the PathTracer ctor
    vector<float> rgb(m->w * m->h * 3);
    for (size_t i = 0; i < m->w * m->h; ++i) {
      rgb[3 * i] = m->data[i].r;
      rgb[3 * i + 1] = m->data[i].g;
      rgb[3 * i + 2] = m->data[i].b;
    }
    w.i8("env_shape", {(int64_t)m->h, (int64_t)m->w});
    w.f4("env_rgb", rgb);
  }

  const vector<StaticScene::Primitive*>& prims = pt.bvh->primitives;
  vector<int32_t> ptype, pbsdf, porig;
  vector<double> pgeom, pnorm;
  for (StaticScene::Primitive* p : prims) {
    ptype.push_back(p->getType());
    pbsdf.push_back(bidx[p->get_bsdf()]);
    porig.push_back(orig[p]);
    double g[9] = {0}, n[9] = {0};
    if (p->getType() == 1) {
      auto* t = static_cast<StaticScene::Triangle*>(p);
      size_t vi[3] = {t->v1, t->v2, t->v3};
      for (int k = 0; k < 3; ++k) {
        const Vector3D& P = t->mesh->positions[vi[k]];
        const Vector3D& N = t->mesh->normals[vi[k]];
        g[3 * k] = P.x; g[3 * k + 1] = P.y; g[3 * k + 2] = P.z;
        n[3 * k] = N.x; n[3 * k + 1] = N.y; n[3 * k + 2] = N.z;
      }
    } else {
      auto* s = static_cast<StaticScene::Sphere*>(p);
      g[0] = s->o.x; g[1] = s->o.y; g[2] = s->o.z; g[3] = s->r;
    }
    pgeom.insert(pgeom.end(), g, g + 9);
    pnorm.insert(pnorm.end(), n, n + 9);
  }
  w.i4("prim_type", ptype);
  w.i4("prim_bsdf", pbsdf);
  w.i4("prim_orig", porig);
  w.f8("prim_geom", pgeom);
  w.f8("prim_norm", pnorm);

  // BVH nodes in pre-order (node, left subtree, right subtree).
  vector<double> nbb;
  vector<int64_t> ninfo;
  std::vector<StaticScene::BVHNode*> order;
  std::map<StaticScene::BVHNode*, int64_t> id;
  std::vector<StaticScene::BVHNode*> st = {pt.bvh->get_root()};
  while (!st.empty()) {
    StaticScene::BVHNode* n = st.back();
    st.pop_back();
    id[n] = (int64_t)order.size();
    order.push_back(n);
    if (n->r) st.push_back(n->r);
    if (n->l) st.push_back(n->l);
  }
  for (StaticScene::BVHNode* n : order) {
    nbb.push_back(n->bb.min.x); nbb.push_back(n->bb.min.y); nbb.push_back(n->bb.min.z);
    nbb.push_back(n->bb.max.x); nbb.push_back(n->bb.max.y); nbb.push_back(n->bb.max.z);
    ninfo.push_back((int64_t)n->start);
    ninfo.push_back((int64_t)n->range);
    ninfo.push_back(n->l ? id[n->l] : -1);
    ninfo.push_back(n->r ? id[n->r] : -1);
  }
  w.f8("node_bb", nbb);
  w.i8("node_info", ninfo);
  w.close();
}

// rays mode: input PTDUMP with "ray_o","ray_d" (f8 n*3) and "ray_maxt" (f8 n).
static void answer_rays(const Opts& o, PathTracer& pt) {
  std::vector<ptdump::Record> recs;
  if (!ptdump::read_all(o.rays_in.c_str(), recs)) die("cannot read rays");
  vector<double> ro, rd, rmax;
  ptdump::get(recs, "ray_o", ro);
  ptdump::get(recs, "ray_d", rd);
  ptdump::get(recs, "ray_maxt", rmax);
  size_t n = rmax.size();
  std::map<const StaticScene::Primitive*, int> bidx;
  for (size_t i = 0; i < pt.bvh->primitives.size(); ++i) bidx[pt.bvh->primitives[i]] = (int)i;
  vector<int32_t> hit(n), prim(n), any(n);
  vector<double> t(n), nrm(3 * n);
  for (size_t i = 0; i < n; ++i) {
    Vector3D O(ro[3 * i], ro[3 * i + 1], ro[3 * i + 2]), D(rd[3 * i], rd[3 * i + 1], rd[3 * i + 2]);
    Ray r(O, D);
    StaticScene::Intersection isect;
    hit[i] = pt.bvh->intersect(r, &isect) ? 1 : 0;
    t[i] = hit[i] ? isect.t : -1.0;
    prim[i] = hit[i] ? bidx[isect.primitive] : -1;
    nrm[3 * i] = isect.n.x; nrm[3 * i + 1] = isect.n.y; nrm[3 * i + 2] = isect.n.z;
    Ray s(O, D);
    s.max_t = rmax[i];
    any[i] = pt.bvh->intersect(s) ? 1 : 0;
  }
  ptdump::Writer w(o.out.c_str());
  w.i4("hit", hit);
  w.f8("t", t);
  w.i4("prim", prim);
  w.f8("n", nrm);
  w.i4("any", any);
}

#ifndef REF_DRIVER_NO_MAIN
int main(int argc, char** argv) {
  Opts o;
  for (int i = 1; i < argc; ++i) {
    string a = argv[i];
    auto nxt = [&]() -> string { if (i + 1 >= argc) die("missing value"); return argv[++i]; };
    if (a == "--mode") o.mode = nxt();
    else if (a == "--out") o.out = nxt();
    else if (a == "--cam") o.cam = nxt();
    else if (a == "--rays") o.rays_in = nxt();
    else if (a == "-w") o.w = std::stoul(nxt());
    else if (a == "-h") o.h = std::stoul(nxt());
    else if (a == "-s") o.spp = std::stoul(nxt());
    else if (a == "-m") o.depth = std::stoul(nxt());
    else if (a == "-l") o.lights = std::stoul(nxt());
    else if (a == "-t") o.threads = std::stoul(nxt());
    else if (a == "--seed") o.seed = (unsigned)std::stoul(nxt());
    else if (a == "--envmap") o.envmap = nxt();
    else if (a == "--in") o.in = nxt();
    else if (a == "--half") o.half = std::stoi(nxt());
    else if (a == "--tile-begin") o.tile_begin = std::stoul(nxt());
    else if (a == "--tile-stride") o.tile_stride = std::max<size_t>(1, std::stoul(nxt()));
    else o.scene = a;
  }
  if (o.mode == "rng") {
    // Which order does UniformGridSampler2D::get_sample (sampler.cpp:14) draw in?
    std::srand(o.seed);
    UniformGridSampler2D g;
    Vector2D s = g.get_sample();
    std::srand(o.seed);
    int r0 = std::rand(), r1 = std::rand();
    std::printf("sample %.17g %.17g\nrand %d %d\n", s.x, s.y, r0, r1);
    return 0;
  }
  if (o.mode == "exr" || o.mode == "exrw") return exr_modes(o);
  if (o.mode == "tocolor") return tocolor_mode(o);
  if (o.scene.empty()) die("no scene");

  PathTracer* pt = setup_pathtracer(o);

  if (o.mode == "dump") {
    dump_scene(o, *pt);
    return 0;
  }
  if (o.mode == "rays") {
    answer_rays(o, *pt);
    return 0;
  }
  if (o.mode == "tiles") {
    // the per-frame state start_raytracing sets up (pathtracer.cpp:192-207),
    // without its worker threads
    pt->continueRaytracing = true;
    pt->sampleBuffer.clear();
    pt->frameBuffer.clear();
    pt->num_tiles_w = pt->sampleBuffer.w / 32 + 1;
    pt->num_tiles_h = pt->sampleBuffer.h / 32 + 1;
    pt->tile_samples.assign(pt->num_tiles_w * pt->num_tiles_h, 0);
    const size_t ntx = (o.w + 31) / 32, nt = ntx * ((o.h + 31) / 32);
    size_t px = 0, n = 0;
    std::vector<size_t> sample;
    for (size_t i = o.tile_begin; i < nt; i += o.tile_stride) {
      const size_t tx = (i % ntx) * 32, ty = (i / ntx) * 32;
      sample.push_back(i);
      px += (std::min(o.w, tx + 32) - tx) * (std::min(o.h, ty + 32) - ty);
      ++n;
    }
    std::srand(o.seed);
    // -t T: T threads popping the sample's tiles from one shared queue and
    // calling raytrace_tile, as the reference's worker_thread does
    // (pathtracer.cpp:613-637; rand() stays the one shared glibc stream)
    std::atomic<size_t> next{0};
    auto worker = [&]() {
      for (size_t k; (k = next.fetch_add(1)) < sample.size();) {
        const size_t i = sample[k];
        pt->raytrace_tile((int)((i % ntx) * 32), (int)((i / ntx) * 32), 32, 32);
      }
    };
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> pool;
    for (size_t t = 1; t < std::max<size_t>(1, o.threads); ++t) pool.emplace_back(worker);
    worker();
    for (auto& th : pool) th.join();
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("{\"render_s\": %.6f, \"pixels\": %zu, \"tiles\": %zu, \"spp\": %zu, \"threads\": %zu}\n", secs, px, n,
                o.spp, std::max<size_t>(1, o.threads));
    return 0;
  }
  // render (main.cpp:170-181 with srand moved next to the render)
  std::srand(o.seed);
  auto t0 = std::chrono::steady_clock::now();
  pt->start_raytracing();
  for (;;) {
    pt->m.lock();
    int st = pt->state;
    pt->m.unlock();
    if (st == PathTracer::DONE) break;
  }
  auto t1 = std::chrono::steady_clock::now();
  for (size_t i = 0; i < pt->numWorkerThreads; ++i) pt->workerThreads[i]->join();
  double secs = std::chrono::duration<double>(t1 - t0).count();
  std::printf("{\"render_s\": %.6f, \"w\": %zu, \"h\": %zu, \"spp\": %zu, \"threads\": %zu}\n", secs, o.w,
              o.h, o.spp, o.threads);
  if (!o.out.empty()) {
    ptdump::Writer w(o.out.c_str());
    vector<float> hdr(o.w * o.h * 3);
    for (size_t i = 0; i < o.w * o.h; ++i) {
      hdr[3 * i] = pt->sampleBuffer.data[i].r;
      hdr[3 * i + 1] = pt->sampleBuffer.data[i].g;
      hdr[3 * i + 2] = pt->sampleBuffer.data[i].b;
    }
    w.f4("hdr", hdr);
    w.f8("render_s", {secs});
    w.i8("shape", {(int64_t)o.h, (int64_t)o.w, 3});
  }
  return 0;
}
#endif  // REF_DRIVER_NO_MAIN
