// oracle/restate.cpp — ORACLE / TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference hot path, written from the reference's
// behaviour (not copied), used as the parity checker for the HIP path:
//   PathTracer::raytrace_tile   src/pathtracer.cpp:585-611
//   PathTracer::raytrace_pixel  src/pathtracer.cpp:555-583
//   PathTracer::trace_ray       src/pathtracer.cpp:407-553
//   Camera::generate_ray        src/camera.cpp:113-129
//   BVHAccel::intersect (x2)    src/bvh.cpp:227-362,  BBox::intersect src/bbox.cpp:10-30
//   Triangle::intersect (x2)    src/static_scene/triangle.cpp:25-104
//   Sphere::test/intersect      src/static_scene/sphere.cpp:10-77
//   AreaLight/Point/Directional/Hemisphere::sample_L  src/static_scene/light.cpp:17-92
//   Diffuse/Mirror/Refraction/Glass/Emission BSDF     src/bsdf.cpp:13-202
//   Uniform/Cosine samplers     src/sampler.cpp:7-55
//   make_coord_space            src/bsdf.cpp:13-30
// Arithmetic mirrors the reference's types and evaluation order (Vector3D in
// double, Spectrum in float, the implicit double->float conversions at the
// Spectrum operators, ::sqrt resolving to the double overload in bsdf.cpp and
// std::fabs(float) in light.cpp), so that with rng_mode=0 it reproduces the reference
// binary (oracle/_ref) bit for bit at -t 1 on the same srand() seed.
// rng_mode=1 swaps std::rand() for the counter-based stream the HIP kernel uses
// (dsgpuraytracing_amd/csrc/pt_rng.h defines the same function), consumed in
// exactly the reference's draw order, so HIP vs restatement is a near-exact
// per-pixel comparison.
//
// The scene comes from a PTDUMP file: the flattened primitives in BVH order plus
// the reference BVH topology (written by oracle/_ref/ref_driver --mode dump or
// by the product's native loader).  Compile exactly like the reference
// (g++ -O3, no -march, no -ffast-math): see oracle/Makefile.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <thread>
#include <vector>

#include "../dsgpuraytracing_amd/csrc/ptdump.h"

namespace rs {

// Diagnostic trace of one pixel (RS_DEBUG_PIXEL=x,y): prints every hit/NEE/bounce.
static int g_dbg_x = -1, g_dbg_y = -1;
static thread_local bool t_dbg = false;
#define RS_DBG(...) \
  do {              \
    if (t_dbg) std::fprintf(stderr, __VA_ARGS__); \
  } while (0)

static const double PI_D = 3.14159265358979323;
static const double EPS_D = 0.00000000001;
static const double EPS_N = 5e-3;
static const double INF_D = std::numeric_limits<double>::infinity();

struct V3 {
  double x = 0, y = 0, z = 0;
  V3() {}
  V3(double a, double b, double c) : x(a), y(b), z(c) {}
  double& operator[](int i) { return (&x)[i]; }
  double operator[](int i) const { return (&x)[i]; }
  V3 operator-() const { return V3(-x, -y, -z); }
  V3 operator+(const V3& v) const { return V3(x + v.x, y + v.y, z + v.z); }
  V3 operator-(const V3& v) const { return V3(x - v.x, y - v.y, z - v.z); }
  V3 operator*(double c) const { return V3(x * c, y * c, z * c); }
  V3 operator/(double c) const {
    const double rc = 1.0 / c;
    return V3(rc * x, rc * y, rc * z);
  }
  void operator+=(const V3& v) { x += v.x; y += v.y; z += v.z; }
  void operator*=(double c) { x *= c; y *= c; z *= c; }
  double norm() const { return std::sqrt(x * x + y * y + z * z); }
  double norm2() const { return x * x + y * y + z * z; }
  V3 unit() const {
    double r = 1. / std::sqrt(x * x + y * y + z * z);
    return V3(r * x, r * y, r * z);
  }
  void normalize() { (*this) *= (1. / norm()); }
};
inline V3 operator*(double c, const V3& v) { return V3(c * v.x, c * v.y, c * v.z); }
inline double dot(const V3& u, const V3& v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
inline V3 cross(const V3& u, const V3& v) {
  return V3(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}

struct Spec {
  float r = 0, g = 0, b = 0;
  Spec() {}
  Spec(float a, float bb, float c) : r(a), g(bb), b(c) {}
  Spec operator+(const Spec& o) const { return Spec(r + o.r, g + o.g, b + o.b); }
  void operator+=(const Spec& o) { r += o.r; g += o.g; b += o.b; }
  Spec operator*(const Spec& o) const { return Spec(r * o.r, g * o.g, b * o.b); }
  Spec operator*(float s) const { return Spec(r * s, g * s, b * s); }
  void operator*=(float s) { r *= s; g *= s; b *= s; }
  float illum() const { return 0.2126f * r + 0.7152f * g + 0.0722f * b; }
};
inline Spec operator*(float s, const Spec& c) { return c * s; }

// Column-major 3x3 as CMU462::Matrix3x3 (entries[j] = column j).
struct M3 {
  V3 c[3];
  V3 mul(const V3& v) const { return v[0] * c[0] + v[1] * c[1] + v[2] * c[2]; }
  M3 T() const {
    M3 B;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) B.c[j][i] = c[i][j];
    return B;
  }
};

void make_coord_space(M3& o2w, const V3& n) {
  V3 z(n.x, n.y, n.z);
  V3 h = z;
  if (std::fabs(h.x) <= std::fabs(h.y) && std::fabs(h.x) <= std::fabs(h.z)) h.x = 1.0;
  else if (std::fabs(h.y) <= std::fabs(h.x) && std::fabs(h.y) <= std::fabs(h.z)) h.y = 1.0;
  else h.z = 1.0;
  z.normalize();
  V3 y = cross(h, z);
  y.normalize();
  V3 x = cross(z, y);
  x.normalize();
  o2w.c[0] = x;
  o2w.c[1] = y;
  o2w.c[2] = z;
}

struct Ray {
  V3 o, d;
  double min_t = 0.0;
  mutable double max_t = INF_D;
  size_t depth = 0;
  Ray(const V3& o_, const V3& d_) : o(o_), d(d_) {}
};

struct Prim {
  int type;  // 0 sphere, 1 triangle (Primitive::getType)
  int bsdf;
  V3 p[3], n[3];
  V3 o;
  double r = 0, r2 = 0;
};
struct Node {
  V3 bmin, bmax;
  int64_t start, range, l, r;
};
struct Bsdf {
  int type;  // 0 diffuse 1 mirror 2 refraction 3 glass 4 emission
  Spec a, t, e;
  float ior, rough;
};
struct Light {
  int type;  // 0 directional 1 hemisphere 2 point 3 area 4 environment
  Spec rad;
  V3 pos, dir, dimx, dimy;
  float area;
};
struct Camera {
  V3 pos;
  M3 c2w;
  double W, H, dist;
};
// EnvironmentLight (src/static_scene/environment_light.cpp:6-203): the map and
// the tables its constructor builds, in its float arithmetic and order.
struct EnvMap {
  int w = 0, h = 0;
  std::vector<Spec> data;                          // HDRImageBuffer, row 0 = +y
  std::vector<std::vector<float>> pThetaPhi, pPhiGivenTheta;
  std::vector<float> pTheta;
  void build() {  // environment_light.cpp:6-48
    pThetaPhi.assign(h, std::vector<float>(w));
    pTheta.assign(h, 0);
    pPhiGivenTheta.assign(h, std::vector<float>(w));
    float C = 0;
    for (int y = 0; y < h; y++) {
      float theta = (y + 0.5) / h * PI_D;
      float sin_theta = ::sin((double)theta);  // ::sin(double): no std overloads visible there
      for (int x = 0; x < w; x++) {
        pThetaPhi[y][x] = data[x + w * y].illum() * sin_theta;
        C += pThetaPhi[y][x];
      }
    }
    for (int y = 0; y < h; y++) {
      for (int x = 0; x < w; x++) {
        pThetaPhi[y][x] /= C;
        pTheta[y] += pThetaPhi[y][x];
      }
      if (pTheta[y] != 0)
        for (int x = 0; x < w; x++) pPhiGivenTheta[y][x] = pThetaPhi[y][x] / pTheta[y];
    }
    for (int y = 0; y < h; y++) {
      if (y > 0) pTheta[y] += pTheta[y - 1];
      for (int x = 0; x < w; x++)
        if (x > 0) pPhiGivenTheta[y][x] += pPhiGivenTheta[y][x - 1];
    }
  }
};

struct Scene {
  EnvMap env;
  std::vector<Prim> prims;
  std::vector<Node> nodes;
  std::vector<Bsdf> bsdfs;
  std::vector<Light> lights;
  Camera cam;
};

struct Isect {
  double t = INF_D;
  int prim = -1;
  V3 n;
};

struct Stats {
  int64_t rays = 0, shadow = 0, nodes = 0, tris = 0, spheres = 0;
};

// ---------------------------------------------------------------- RNG
// Counter-based stream keyed by (seed, pixel, sample); draw k -> 24-bit uniform.
static inline uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
struct Rng {
  int mode = 0;  // 0: glibc std::rand()/RAND_MAX, 1: counter stream
  uint32_t base = 0, dim = 0;
  void start(uint32_t seed, uint32_t pixel, uint32_t sample) {
    uint32_t h = lowbias32(seed * 0x9E3779B9U ^ pixel);
    base = lowbias32(h ^ (sample * 0x85EBCA6BU));
    dim = 0;
  }
  // rand()/(float)RAND_MAX (environment_light.cpp:67-68): float division
  float next_f() {
    if (mode == 0) return std::rand() / (float)RAND_MAX;
    uint32_t h = lowbias32(base ^ ((dim++) * 0xC2B2AE35U + 0x27D4EB2FU));
    return (float)(h >> 8) * (1.0f / 16777216.0f);
  }
  double next() {
    if (mode == 0) return std::rand() / (double)RAND_MAX;
    uint32_t h = lowbias32(base ^ ((dim++) * 0xC2B2AE35U + 0x27D4EB2FU));
    return (double)(h >> 8) * (1.0 / 16777216.0);
  }
};

// ---------------------------------------------------------------- geometry
static bool bbox_hit(const Node& nd, const Ray& r, double& t0, double& t1) {
  for (int i = 0; i < 3; i++) {
    if (r.d[i] != 0.0) {
      double tx1 = (nd.bmin[i] - r.o[i]) / r.d[i];
      double tx2 = (nd.bmax[i] - r.o[i]) / r.d[i];
      t0 = std::max(t0, std::min(tx1, tx2));
      t1 = std::min(t1, std::max(tx1, tx2));
    }
  }
  return t0 <= t1;
}

static bool tri_hit(const Prim& P, const Ray& r, Isect* is, Stats& st) {
  st.tris++;
  V3 e1 = P.p[1] - P.p[0];
  V3 e2 = P.p[2] - P.p[0];
  V3 s = r.o - P.p[0];
  double f = dot(cross(e1, r.d), e2);
  if (f == 0) return false;
  double u = dot(cross(s, r.d), e2) / f;
  double v = dot(cross(e1, r.d), s) / f;
  double t = dot(cross(e1, -s), e2) / f;
  if (!is) return u >= 0 && v >= 0 && u + v <= 1 && t > r.min_t && t < r.max_t;
  if (!(u >= 0 && v >= 0 && u + v <= 1 && t > r.min_t && t < r.max_t && t < is->t)) return false;
  r.max_t = t;
  is->t = t;
  V3 n = (1 - u - v) * P.n[0] + u * P.n[1] + v * P.n[2];
  if (dot(r.d, n) > 0) n = -n;
  is->n = n;
  return true;
}

static bool sphere_test(const Prim& P, const Ray& r, double& t1, double& t2) {
  V3 m = P.o - r.o;
  double b = dot(m, r.d);
  double c = dot(m, m) - P.r2;
  double delta = b * b - c;
  if (delta < 0) return false;
  t1 = b - std::sqrt(delta);
  t2 = b + std::sqrt(delta);
  if (t1 >= r.max_t || t2 <= r.min_t) return false;
  return true;
}

static bool sphere_test_alias(const Prim& P, const Ray& r, double& t) {
  V3 m = P.o - r.o;
  double b = dot(m, r.d);
  double c = dot(m, m) - P.r2;
  double delta = b * b - c;
  if (delta < 0) return false;
  t = b - std::sqrt(delta);
  t = b + std::sqrt(delta);
  if (t >= r.max_t || t <= r.min_t) return false;
  return true;
}

static bool sphere_hit(const Prim& P, const Ray& r, Isect* is, Stats& st) {
  st.spheres++;
  double t1, t2;
  // Sphere::intersect(r) (sphere.cpp:37-45) calls test(r, tmp, tmp): both
  // out-references alias one double, so the range check sees the far root twice.
  if (!is) {
    double tmp;
    if (!sphere_test_alias(P, r, tmp)) return false;
    return true;
  }
  if (!sphere_test(P, r, t1, t2)) return false;
  double t = t1;
  if (t1 <= r.min_t) t = t2;
  V3 n = r.o + r.d * t - P.o;
  n.normalize();
  is->n = n;
  is->t = t;
  r.max_t = t;
  return true;
}

struct Tracer {
  const Scene& S;
  Stats st;
  explicit Tracer(const Scene& s) : S(s) {}

  bool prim_hit(int64_t i, const Ray& r, Isect* is) {
    const Prim& P = S.prims[i];
    bool h = P.type == 1 ? tri_hit(P, r, is, st) : sphere_hit(P, r, is, st);
    if (h && is) is->prim = (int)i;
    return h;
  }

  // bvh.cpp:227-279 (nearest) and 282-329 (any); same visit order and pruning.
  bool node_isect(int64_t ni, const Ray& ray, Isect* is) {
    st.nodes++;
    const Node& nd = S.nodes[ni];
    if (nd.l < 0 && nd.r < 0) {
      bool any = false;
      for (int64_t j = 0; j < nd.range; j++) {
        bool res = prim_hit(j + nd.start, ray, is);
        if (!is && res) return true;
        any = any || res;
      }
      return any;
    }
    if (nd.l < 0) return node_isect(nd.r, ray, is);
    if (nd.r < 0) return node_isect(nd.l, ray, is);
    double tminl = -INF_D, tminr = -INF_D, tmaxl = INF_D, tmaxr = INF_D;
    Ray nray = ray;
    nray.d += V3(EPS_D, EPS_D, EPS_D);
    nray.d.normalize();
    bool hitl = bbox_hit(S.nodes[nd.l], nray, tminl, tmaxl);
    bool hitr = bbox_hit(S.nodes[nd.r], nray, tminr, tmaxr);
    if (hitl && hitr) {
      int64_t first = (tminl <= tminr) ? nd.l : nd.r;
      int64_t second = (tminl <= tminr) ? nd.r : nd.l;
      if (!is) return node_isect(first, ray, is) || node_isect(second, ray, is);
      hitl = node_isect(first, ray, is);
      if (!hitl || is->t > std::max(tminl, tminr)) hitr = node_isect(second, ray, is);
      return hitl || hitr;
    } else if (hitl) {
      return node_isect(nd.l, ray, is);
    } else if (hitr) {
      return node_isect(nd.r, ray, is);
    }
    return false;
  }
  bool intersect(const Ray& r, Isect* is) { return node_isect(0, r, is); }

  // EnvironmentLight::sample_dir (environment_light.cpp:130-199)
  Spec env_dir(const V3& d) const {
    const EnvMap& E = S.env;
    const int w = E.w, h = E.h;
    double theta = ::acos(d[1]);
    double sin_theta = ::sqrt(1 - d[1] * d[1]);
    double phi = sin_theta == 0 ? PI_D : ::acos(std::min(std::max(d[2] / sin_theta, -1.0), 1.0));
    if (d[0] > 0) phi = 2 * PI_D - phi;
    double u = phi / (2 * PI_D);
    double v = theta / PI_D;
    float tu = u * w - 0.5;
    float tv = v * h - 0.5;
    int su = (int)tu;
    int sv = (int)tv;
    float a, b;
    int px1, px2, py1, py2;
    if (tu < 0) {
      a = tu + 1; px1 = w - 1; px2 = 0;
    } else if (tu >= w - 1) {
      a = tu - w + 1; px1 = w - 1; px2 = 0;
    } else {
      a = tu - su; px1 = su; px2 = su + 1;
    }
    if (tv < 0) {
      b = tv + 1; py1 = h - 1; py2 = 0;
    } else if (tv >= h - 1) {
      b = tv - h + 1; py1 = h - 1; py2 = 0;
    } else {
      b = tv - sv; py1 = sv; py2 = sv + 1;
    }
    Spec z11 = E.data[px1 + w * py1], z21 = E.data[px2 + w * py1];
    Spec z12 = E.data[px1 + w * py2], z22 = E.data[px2 + w * py2];
    Spec zy1 = z11 * (1 - a) + z21 * a;
    Spec zy2 = z12 * (1 - a) + z22 * a;
    return zy1 * (1 - b) + zy2 * b;
  }

  // EnvironmentLight::importanceSampling (environment_light.cpp:69-115)
  void env_importance(V3* wi, float* pdf, Rng& rng) const {
    const EnvMap& E = S.env;
    float r1 = rng.next_f();
    float r2 = rng.next_f();
    r1 *= E.pTheta.back();
    auto itr = std::lower_bound(E.pTheta.begin(), E.pTheta.end(), r1);
    int t = (int)(itr - E.pTheta.begin());
    float prev = t > 0 ? *(itr - 1) : 0;
    float y = t + (r1 - prev) / (*itr - prev);
    float theta = std::min(y / E.h, 1.f) * PI_D;
    const std::vector<float>& row = E.pPhiGivenTheta[t];
    r2 *= row.back();
    itr = std::lower_bound(row.begin(), row.end(), r2);
    int q = (int)(itr - row.begin());
    prev = q > 0 ? *(itr - 1) : 0;
    float x = q + (r2 - prev) / (*itr - prev);
    float phi = std::min(x / E.w, 1.f) * 2 * PI_D;
    double sin_theta = ::sin((double)theta);
    double cos_theta = ::cos((double)theta);
    *pdf = E.pThetaPhi[t][q];
    *pdf /= (sin_theta * (2 * PI_D / E.w) * (PI_D / E.h));
    *wi = V3(-sin_theta * ::sin((double)phi), cos_theta, sin_theta * ::cos((double)phi));
  }

  // light.cpp:17-92
  Spec sample_L(const Light& L, const V3& p, V3* wi, float* dist, float* pdf, Rng& rng) {
    if (L.type == 4) {  // EnvironmentLight::sample_L (environment_light.cpp:117-128)
      env_importance(wi, pdf, rng);
      *dist = (float)INF_D;
      return env_dir(*wi);
    }
    if (L.type == 0) {
      *wi = L.dir;
      *dist = (float)INF_D;
      *pdf = 1.0;
      return L.rad;
    }
    if (L.type == 1) {
      double r1 = rng.next();
      double r2 = rng.next();
      double sin_theta = std::sqrt(1 - r1 * r1);
      double phi = 2 * PI_D * r2;
      V3 dir(sin_theta * std::cos(phi), sin_theta * std::sin(phi), r1);
      M3 s2w;
      s2w.c[0] = V3(1, 0, 0);
      s2w.c[1] = V3(0, 0, -1);
      s2w.c[2] = V3(0, 1, 0);
      *wi = s2w.mul(dir);
      *dist = (float)INF_D;
      *pdf = 1.0 / (2.0 * M_PI);
      return L.rad;
    }
    if (L.type == 2) {
      V3 d = L.pos - p;
      *wi = d.unit();
      *dist = d.norm();
      *pdf = 1.0;
      return L.rad;
    }
    // Area light. UniformGridSampler2D::get_sample evaluates its two rand()
    // arguments right to left under g++: the FIRST draw is y.
    double sy = rng.next();
    double sx = rng.next();
    sx = sx - 0.5f;
    sy = sy - 0.5f;
    V3 d = L.pos + sx * L.dimx + sy * L.dimy - p;
    float cosTheta = dot(d, L.dir);
    float sqDist = d.norm2();
    float dst = ::sqrt((double)sqDist);
    *wi = d / dst;
    *dist = dst;
    // light.cpp sees `using namespace std` (via its headers): fabs(float) is
    // std::fabs(float), so the pdf is computed entirely in float.
    *pdf = sqDist / (L.area * std::fabs(cosTheta));
    return cosTheta < 0 ? L.rad : Spec();
  }

  static bool is_delta(const Bsdf& b) { return b.type == 1 || b.type == 2 || b.type == 3; }

  static Spec f(const Bsdf& b) {
    if (b.type == 0) return b.a * (float)(1.0 / PI_D);
    return Spec();
  }

  static bool refract(const V3& wo, V3* wi, float ior) {
    int sign = 1;
    float ratio = ior;
    if (wo[2] > 0) {
      sign = -1;
      ratio = 1 / ratio;
    }
    float cos2_wi = 1 - ratio * ratio * (1 - wo[2] * wo[2]);
    if (cos2_wi < 0) {
      *wi = V3(-wo[0], -wo[1], wo[2]);
      return false;
    }
    *wi = V3(-wo[0] * ratio, -wo[1] * ratio, sign * ::sqrt((double)cos2_wi)).unit();
    return true;
  }

  static V3 cosine_sample(float* pdf, Rng& rng) {
    double r1 = rng.next();
    double r2 = rng.next();
    double theta = std::acos(1 - 2 * r1) / 2;
    double phi = 2 * PI_D * r2;
    double sin_theta = std::sin(theta);
    double cos_theta = std::cos(theta);
    *pdf = cos_theta / PI_D;
    return V3(sin_theta * std::cos(phi), sin_theta * std::sin(phi), cos_theta);
  }

  Spec sample_f(const Bsdf& b, const V3& wo, V3* wi, float* pdf, Rng& rng) {
    switch (b.type) {
      case 0:
        *wi = cosine_sample(pdf, rng);
        return b.a * (float)(1.0 / PI_D);
      case 1:
        *wi = V3(-wo[0], -wo[1], wo[2]);
        *pdf = 1;
        return b.a * (float)(1 / std::max(wo[2], 1e-8));
      case 2: {
        *pdf = 1;
        if (!refract(wo, wi, b.ior)) return Spec();
        double ni = b.ior, no = 1;
        if (wo[2] < 0) std::swap(ni, no);
        double ratio = no / ni;
        // bsdf.cpp:110 `transmittance * ratio*ratio * (...)`: three float products
        return b.t * (float)ratio * (float)ratio * (float)(1 / std::max(std::fabs((*wi)[2]), 1e-8));
      }
      case 3: {
        *pdf = 1;
        if (!refract(wo, wi, b.ior)) return b.t * (float)(1 / std::max(std::fabs((*wi)[2]), 1e-8));
        double ni = b.ior, no = 1;
        double cos_i = std::fabs((*wi)[2]);
        double cos_o = std::fabs(wo[2]);
        if (wo[2] < 0) std::swap(ni, no);
        double r1 = (no * cos_i - ni * cos_o) / (no * cos_i + ni * cos_o);
        double r2 = (ni * cos_i - no * cos_o) / (ni * cos_i + no * cos_o);
        double Fr = 0.5 * (r1 * r1 + r2 * r2);
        if (rng.next() <= Fr) {
          *wi = V3(-wo[0], -wo[1], wo[2]);
          return b.a * (float)(1 / std::max(std::fabs((*wi)[2]), 1e-8));
        }
        double ratio = no / ni;
        return b.t * (float)ratio * (float)ratio * (float)(1 / std::max(std::fabs((*wi)[2]), 1e-8));
      }
      default:
        *wi = cosine_sample(pdf, rng);
        return Spec();
    }
  }

  int max_depth = 4, ns_area_light = 1;

  // pathtracer.cpp:407-553
  Spec trace_ray(const Ray& r, bool includeLe, Rng& rng) {
    st.rays++;
    Isect isect;
    if (!intersect(r, &isect)) {  // pathtracer.cpp:411-427
      if (S.env.w > 0 && includeLe) return env_dir(r.d);
      return Spec(0, 0, 0);
    }
    const Prim& P = S.prims[isect.prim];
    const Bsdf& B = S.bsdfs[P.bsdf];
    RS_DBG("  depth %zu hit prim %d (type %d bsdf %d) t=%.9g n=(%.6g %.6g %.6g)\n", r.depth, isect.prim, P.type,
           P.bsdf, isect.t, isect.n.x, isect.n.y, isect.n.z);
    Spec L_out = includeLe ? B.e : Spec();
    V3 hit_p = r.o + r.d * isect.t;
    M3 o2w;
    make_coord_space(o2w, isect.n);
    M3 w2o = o2w.T();
    V3 w_out = w2o.mul(r.o - hit_p);
    w_out.normalize();
    V3 dir_to_light;
    float dist_to_light;
    float pdf;
    for (const Light& light : S.lights) {
      Spec L(0, 0, 0);
      bool delta = light.type == 0 || light.type == 2;
      int num_light_samples = delta ? 1 : ns_area_light;
      double scale = 1.0 / num_light_samples;
      for (int i = 0; i < num_light_samples; i++) {
        Spec light_L = sample_L(light, hit_p, &dir_to_light, &dist_to_light, &pdf, rng);
        double eps = delta ? EPS_N : 0;
        Ray sR(hit_p + eps * isect.n + EPS_D * dir_to_light, dir_to_light);
        sR.max_t = dist_to_light * 0.999;
        st.shadow++;
        if (intersect(sR, nullptr)) {
          RS_DBG("    shadow ray occluded (Li %.4g pdf %.4g dist %.6g)\n", light_L.r, pdf, dist_to_light);
          continue;
        }
        V3 w_in = w2o.mul(dir_to_light);
        w_in.normalize();
        double cos_theta = std::max(0.0, w_in[2]);
        Spec fv = f(B);
        L += (float)(cos_theta / pdf) * light_L * fv;
        RS_DBG("    shadow o=(%.9g %.9g %.9g) d=(%.9g %.9g %.9g) maxt=%.9g\n", sR.o.x, sR.o.y, sR.o.z, sR.d.x, sR.d.y,
               sR.d.z, sR.max_t);
        RS_DBG("    NEE + %.6g (cos %.4g pdf %.4g Li %.4g)\n", (float)(cos_theta / pdf) * light_L.r * fv.r, cos_theta,
               pdf, light_L.r);
      }
      L_out += L * (float)scale;
    }
    if (r.depth >= (size_t)max_depth) return L_out;
    V3 w_in;
    Spec fs = sample_f(B, w_out, &w_in, &pdf, rng);
    double cos_theta = std::fabs(w_in[2]);
    double terminateProbability = std::max(1 - fs.illum(), 0.f);
    if (rng.next() < terminateProbability) {
      RS_DBG("    RR terminate (p=%.4g)\n", terminateProbability);
      return L_out;
    }
    RS_DBG("    bounce wi=(%.6g %.6g %.6g) pdf %.5g p %.4g\n", w_in.x, w_in.y, w_in.z, pdf, terminateProbability);
    V3 v = o2w.mul(w_in);
    v.normalize();
    Ray refR(hit_p + EPS_D * v, v);
    refR.depth = r.depth + 1;
    Spec indirL = trace_ray(refR, is_delta(B), rng);
    return L_out + (float)(cos_theta / (pdf * (1 - terminateProbability))) * indirL * fs;
  }

  Ray generate_ray(double x, double y) const {
    const Camera& c = S.cam;
    V3 sp(-(x - 0.5) * c.W / c.dist, -(y - 0.5) * c.H / c.dist, 1);
    V3 dir = -sp;
    V3 world_sp = c.c2w.mul(sp) + c.pos;
    V3 world_dir = c.c2w.mul(dir);
    world_dir.normalize();
    return Ray(world_sp, world_dir);
  }
};

static bool load_scene(const char* path, Scene& S) {
  std::vector<ptdump::Record> R;
  if (!ptdump::read_all(path, R)) return false;
  std::vector<double> cam, lgeom, pgeom, pnorm, nbb;
  std::vector<float> bpar, lrad, larea;
  std::vector<int32_t> btype, ltype, ptype, pbsdf;
  std::vector<int64_t> ninfo;
  bool ok = ptdump::get(R, "cam", cam) && ptdump::get(R, "bsdf_type", btype) &&
            ptdump::get(R, "bsdf_params", bpar) && ptdump::get(R, "light_type", ltype) &&
            ptdump::get(R, "light_rad", lrad) && ptdump::get(R, "light_geom", lgeom) &&
            ptdump::get(R, "light_area", larea) && ptdump::get(R, "prim_type", ptype) &&
            ptdump::get(R, "prim_bsdf", pbsdf) && ptdump::get(R, "prim_geom", pgeom) &&
            ptdump::get(R, "prim_norm", pnorm) && ptdump::get(R, "node_bb", nbb) &&
            ptdump::get(R, "node_info", ninfo);
  if (!ok || cam.size() < 15) return false;
  S.cam.pos = V3(cam[0], cam[1], cam[2]);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) S.cam.c2w.c[j][i] = cam[3 + 3 * i + j];
  S.cam.W = cam[12];
  S.cam.H = cam[13];
  S.cam.dist = cam[14];
  S.bsdfs.resize(btype.size());
  for (size_t i = 0; i < btype.size(); ++i) {
    const float* p = &bpar[12 * i];
    Bsdf& b = S.bsdfs[i];
    b.type = btype[i];
    b.a = Spec(p[0], p[1], p[2]);
    b.t = Spec(p[3], p[4], p[5]);
    b.e = Spec(p[6], p[7], p[8]);
    b.ior = p[9];
    b.rough = p[10];
  }
  {
    std::vector<int64_t> eshape;
    std::vector<float> ergb;
    if (ptdump::get(R, "env_shape", eshape) && ptdump::get(R, "env_rgb", ergb) && eshape.size() == 2) {
      S.env.h = (int)eshape[0];
      S.env.w = (int)eshape[1];
      S.env.data.resize((size_t)S.env.w * S.env.h);
      for (size_t i = 0; i < S.env.data.size(); ++i) S.env.data[i] = Spec(ergb[3 * i], ergb[3 * i + 1], ergb[3 * i + 2]);
      S.env.build();
    }
  }
  S.lights.resize(ltype.size());
  for (size_t i = 0; i < ltype.size(); ++i) {
    Light& L = S.lights[i];
    const double* g = &lgeom[12 * i];
    L.type = ltype[i];
    L.rad = Spec(lrad[3 * i], lrad[3 * i + 1], lrad[3 * i + 2]);
    L.pos = V3(g[0], g[1], g[2]);
    L.dir = V3(g[3], g[4], g[5]);
    L.dimx = V3(g[6], g[7], g[8]);
    L.dimy = V3(g[9], g[10], g[11]);
    L.area = larea[i];
  }
  S.prims.resize(ptype.size());
  for (size_t i = 0; i < ptype.size(); ++i) {
    Prim& P = S.prims[i];
    P.type = ptype[i];
    P.bsdf = pbsdf[i];
    const double* g = &pgeom[9 * i];
    const double* n = &pnorm[9 * i];
    for (int k = 0; k < 3; ++k) {
      P.p[k] = V3(g[3 * k], g[3 * k + 1], g[3 * k + 2]);
      P.n[k] = V3(n[3 * k], n[3 * k + 1], n[3 * k + 2]);
    }
    if (P.type == 0) {
      P.o = P.p[0];
      P.r = g[3];
      P.r2 = P.r * P.r;
    }
  }
  size_t nn = nbb.size() / 6;
  S.nodes.resize(nn);
  for (size_t i = 0; i < nn; ++i) {
    Node& N = S.nodes[i];
    N.bmin = V3(nbb[6 * i], nbb[6 * i + 1], nbb[6 * i + 2]);
    N.bmax = V3(nbb[6 * i + 3], nbb[6 * i + 4], nbb[6 * i + 5]);
    N.start = ninfo[4 * i];
    N.range = ninfo[4 * i + 1];
    N.l = ninfo[4 * i + 2];
    N.r = ninfo[4 * i + 3];
  }
  return nn > 0;
}

}  // namespace rs

extern "C" {

// Renders tiles [tile_begin, tile_end) of the reference's row-major 32x32 tile
// FIFO (pathtracer.cpp:210-214) into hdr_out (float32 W*H*3, y=0 bottom).
// rng_mode 0: glibc rand() after srand(seed), single thread, reference order.
// rng_mode 1: counter stream, `threads` workers over tiles.
// stats_out (nullable): rays, shadow rays, node visits, tri tests, sphere tests.
// rs_render_strided: tiles tile_begin, tile_begin + stride, ... < tile_end
// (a uniform sample of the frame for the bench's CPU baseline); render_s
// (nullable) receives the wall time of the render alone (scene load excluded).
int rs_render_strided(const char* scene_path, int w, int h, int spp, int max_depth, int ns_area_light,
                      uint32_t seed, int rng_mode, int threads, int tile_begin, int tile_end, int tile_stride,
                      float* hdr_out, int64_t* stats_out, double* render_s);

int rs_render(const char* scene_path, int w, int h, int spp, int max_depth, int ns_area_light,
              uint32_t seed, int rng_mode, int threads, int tile_begin, int tile_end, float* hdr_out,
              int64_t* stats_out) {
  return rs_render_strided(scene_path, w, h, spp, max_depth, ns_area_light, seed, rng_mode, threads, tile_begin,
                           tile_end, 1, hdr_out, stats_out, nullptr);
}

int rs_render_strided(const char* scene_path, int w, int h, int spp, int max_depth, int ns_area_light,
                      uint32_t seed, int rng_mode, int threads, int tile_begin, int tile_end, int tile_stride,
                      float* hdr_out, int64_t* stats_out, double* render_s) {
  rs::Scene S;
  if (!rs::load_scene(scene_path, S)) return -1;
  if (tile_stride < 1) tile_stride = 1;
  const auto t_start = std::chrono::steady_clock::now();
  const int T = 32;
  std::vector<std::pair<int, int>> tiles;
  for (int y = 0; y < h; y += T)
    for (int x = 0; x < w; x += T) tiles.push_back({x, y});
  if (tile_end < 0 || tile_end > (int)tiles.size()) tile_end = (int)tiles.size();
  if (tile_begin < 0) tile_begin = 0;
  if (const char* dp = std::getenv("RS_DEBUG_PIXEL")) std::sscanf(dp, "%d,%d", &rs::g_dbg_x, &rs::g_dbg_y);
  std::atomic<int> next(tile_begin);
  std::vector<rs::Stats> stats(std::max(1, threads));
  auto worker = [&](int wid) {
    rs::Tracer tr(S);
    tr.max_depth = max_depth;
    tr.ns_area_light = ns_area_light;
    rs::Rng rng;
    rng.mode = rng_mode;
    for (;;) {
      int ti = next.fetch_add(tile_stride);
      if (ti >= tile_end) break;
      int x0 = tiles[ti].first, y0 = tiles[ti].second;
      int x1 = std::min(x0 + T, w), y1 = std::min(y0 + T, h);
      for (int y = y0; y < y1; y++) {
        for (int x = x0; x < x1; x++) {
          rs::Spec s(0, 0, 0);
          uint32_t pix = (uint32_t)(x + y * w);
          rs::t_dbg = (x == rs::g_dbg_x && y == rs::g_dbg_y);
          for (int i = 0; i < spp; i++) {
            if (rng_mode == 1) rng.start(seed, pix, (uint32_t)i);
            if (rs::t_dbg) std::fprintf(stderr, "pixel (%d,%d) sample %d\n", x, y, i);
            double ry = rng.next();  // UniformGridSampler2D: right-to-left
            double rx = rng.next();
            double px = (x + rx) / w;
            double py = (y + ry) / h;
            rs::Ray r = tr.generate_ray(px, py);
            s += tr.trace_ray(r, true, rng);
          }
          s *= (float)(1.0 / spp);
          float* o = hdr_out + 3 * (size_t)pix;
          o[0] = s.r;
          o[1] = s.g;
          o[2] = s.b;
        }
      }
    }
    stats[wid] = tr.st;
  };
  if (rng_mode == 0) {
    std::srand(seed);
    worker(0);
  } else {
    int nt = std::max(1, threads);
    std::vector<std::thread> th;
    for (int i = 0; i < nt; ++i) th.emplace_back(worker, i);
    for (auto& t : th) t.join();
  }
  if (render_s) *render_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
  if (stats_out) {
    int64_t a[5] = {0, 0, 0, 0, 0};
    for (auto& s : stats) {
      a[0] += s.rays; a[1] += s.shadow; a[2] += s.nodes; a[3] += s.tris; a[4] += s.spheres;
    }
    for (int i = 0; i < 5; ++i) stats_out[i] = a[i];
  }
  return 0;
}

// Each sample's radiance of the listed pixels, counter RNG (raytrace_pixel's
// loop, pathtracer.cpp:571-577, without the average): out[(k*spp + i)*3] is
// sample i of pixel (xs[k], ys[k]).  For tools/silhouette_samples.py: which
// samples of a pixel the HIP path and the restatement disagree on.
int rs_pixel_samples(const char* scene_path, int w, int h, int spp, int max_depth, int ns_area_light,
                     uint32_t seed, int n_px, const int32_t* xs, const int32_t* ys, float* out) {
  rs::Scene S;
  if (!rs::load_scene(scene_path, S)) return -1;
  rs::Tracer tr(S);
  tr.max_depth = max_depth;
  tr.ns_area_light = ns_area_light;
  rs::Rng rng;
  rng.mode = 1;
  for (int k = 0; k < n_px; ++k) {
    const int x = xs[k], y = ys[k];
    for (int i = 0; i < spp; i++) {
      rng.start(seed, (uint32_t)(x + y * w), (uint32_t)i);
      double ry = rng.next();
      double rx = rng.next();
      rs::Ray r = tr.generate_ray((x + rx) / w, (y + ry) / h);
      rs::Spec s = tr.trace_ray(r, true, rng);
      float* o = out + 3 * ((size_t)k * spp + i);
      o[0] = s.r;
      o[1] = s.g;
      o[2] = s.b;
    }
  }
  return 0;
}

// BVHAccel::intersect nearest (hit,t,prim,n) and any-hit under max_t (any).
int rs_intersect(const char* scene_path, int64_t n, const double* o, const double* d,
                 const double* maxt, int32_t* hit, double* t, int32_t* prim, double* nrm,
                 int32_t* any) {
  rs::Scene S;
  if (!rs::load_scene(scene_path, S)) return -1;
  rs::Tracer tr(S);
  for (int64_t i = 0; i < n; ++i) {
    rs::V3 O(o[3 * i], o[3 * i + 1], o[3 * i + 2]), D(d[3 * i], d[3 * i + 1], d[3 * i + 2]);
    rs::Ray r(O, D);
    rs::Isect is;
    bool h = tr.intersect(r, &is);
    hit[i] = h;
    t[i] = h ? is.t : -1.0;
    prim[i] = h ? is.prim : -1;
    nrm[3 * i] = is.n.x;
    nrm[3 * i + 1] = is.n.y;
    nrm[3 * i + 2] = is.n.z;
    rs::Ray s(O, D);
    s.max_t = maxt[i];
    any[i] = tr.intersect(s, nullptr);
  }
  return 0;
}

// The counter RNG, exposed so tests can pin the HIP copy (pt_rng.h) against it.
double rs_rng_draw(uint32_t seed, uint32_t pixel, uint32_t sample, uint32_t k) {
  rs::Rng r;
  r.mode = 1;
  r.start(seed, pixel, sample);
  double v = 0;
  for (uint32_t i = 0; i <= k; ++i) v = r.next();
  return v;
}
}
