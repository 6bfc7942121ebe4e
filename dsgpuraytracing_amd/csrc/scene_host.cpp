// scene_host.cpp — native host scene pipeline (include/ptgpu_scene.h).
//
// Produces the flattened scene the GPU seam consumes, bit-identical to what the
// reference's own host code builds (pinned by tests/test_scene_loader.py
// against dumps written by the reference).  Restated, not copied:
//   * a minimal XML reader (the reference uses vendored tinyxml2);
//   * ColladaParser semantics (src/collada/collada.cpp): up-axis correction
//     (162-201), node transforms incl. their quirks (234-328: zero-initialised
//     rotate/translate/scale matrices, children pushed before parents),
//     camera/light/sphere/polylist/material parsing (430-936);
//   * Application::load (src/application.cpp:223-299) camera placement;
//   * DynamicScene::{Mesh,Sphere,AreaLight,...} -> StaticScene conversion;
//   * HalfedgeMesh::build (src/halfEdgeMesh.cpp:29-397) connectivity, vertex
//     order and Vertex::computeNormal (src/halfEdgeMesh.h:492-515);
//   * StaticScene::Mesh triangle order (src/static_scene/object.cpp:16-58);
//   * buildBVH (src/bvh.cpp:21-202) binned SAH, 32 buckets, leaf <= 4, with
//     the bucket index clamped.
// Arithmetic keeps the reference's types (double vectors, float spectra/fov)
// and evaluation order so results match to the last bit.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <string>
#include <utility>
#include <vector>

#include "../../include/ptgpu.h"
#include "../../include/ptgpu_scene.h"
#include "pt_error.h"
#include "ptdump.h"

namespace hs {

static const double PI_D = 3.14159265358979323;
static const double INF_D = std::numeric_limits<double>::infinity();
static const float EPS_F = 0.00001f;

// ------------------------------------------------------------------ math
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
  V3 unit() const {
    double r = 1. / std::sqrt(x * x + y * y + z * z);
    return V3(r * x, r * y, r * z);
  }
  void normalize() { (*this) *= (1. / norm()); }
};
inline V3 operator*(double c, const V3& v) { return V3(c * v.x, c * v.y, c * v.z); }
inline V3 cross(const V3& u, const V3& v) {
  return V3(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}

struct V4 {
  double x = 0, y = 0, z = 0, w = 0;
  V4() {}
  V4(double a, double b, double c, double d) : x(a), y(b), z(c), w(d) {}
  V4(const V3& v, double d) : x(v.x), y(v.y), z(v.z), w(d) {}
  double operator[](int i) const { return (&x)[i]; }
  V4 operator+(const V4& v) const { return V4(x + v.x, y + v.y, z + v.z, w + v.w); }
  V3 to3D() const { return V3(x, y, z); }
  V3 projectTo3D() const {
    double invW = 1.0 / w;
    return V3(x * invW, y * invW, z * invW);
  }
};
inline V4 operator*(double c, const V4& v) { return V4(c * v.x, c * v.y, c * v.z, c * v.w); }

// Column-major 4x4 (CMU462::Matrix4x4: entries[j] = column j, default = zero).
struct M4 {
  V4 col[4];
  double& at(int i, int j) { return (&col[j].x)[i]; }
  double at(int i, int j) const { return (&col[j].x)[i]; }
  static M4 identity() {
    M4 B;
    for (int i = 0; i < 4; ++i) B.at(i, i) = 1.;
    return B;
  }
  M4 operator*(const M4& B) const {
    M4 C;
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < 4; j++) {
        C.at(i, j) = 0.;
        for (int k = 0; k < 4; k++) C.at(i, j) += at(i, k) * B.at(k, j);
      }
    return C;
  }
  V4 operator*(const V4& v) const { return v[0] * col[0] + v[1] * col[1] + v[2] * col[2] + v[3] * col[3]; }
};

struct BBox {
  V3 max = V3(-INF_D, -INF_D, -INF_D), min = V3(INF_D, INF_D, INF_D), extent;
  BBox() { extent = max - min; }
  BBox(const V3& mn, const V3& mx) : max(mx), min(mn) { extent = max - min; }
  void expand(const BBox& b) {
    min.x = std::min(min.x, b.min.x);
    min.y = std::min(min.y, b.min.y);
    min.z = std::min(min.z, b.min.z);
    max.x = std::max(max.x, b.max.x);
    max.y = std::max(max.y, b.max.y);
    max.z = std::max(max.z, b.max.z);
    extent = max - min;
  }
  void expand(const V3& p) {
    min.x = std::min(min.x, p.x);
    min.y = std::min(min.y, p.y);
    min.z = std::min(min.z, p.z);
    max.x = std::max(max.x, p.x);
    max.y = std::max(max.y, p.y);
    max.z = std::max(max.z, p.z);
    extent = max - min;
  }
  V3 centroid() const { return (min + max) / 2; }
  bool empty() const { return min.x > max.x || min.y > max.y || min.z > max.z; }
};

template <typename T>
inline T radians(T deg) { return deg * (PI_D / 180); }
template <typename T>
inline T degrees(T rad) { return rad * (180 / PI_D); }

// ------------------------------------------------------------------ XML
struct XNode {
  std::string name;
  std::vector<std::pair<std::string, std::string>> attrs;
  std::string text;  // first child if it is a text node (tinyxml2 GetText)
  bool has_text = false;
  std::vector<XNode*> kids;
  XNode* parent = nullptr;
  const char* attr(const char* k) const {
    for (auto& a : attrs)
      if (a.first == k) return a.second.c_str();
    return nullptr;
  }
  XNode* first(const std::string& n) const {
    for (XNode* c : kids)
      if (n.empty() || c->name == n) return c;
    return nullptr;
  }
  XNode* next_sibling(const std::string& n) const {
    if (!parent) return nullptr;
    auto& v = parent->kids;
    auto it = std::find(v.begin(), v.end(), this);
    for (++it; it != v.end(); ++it)
      if (n.empty() || (*it)->name == n) return *it;
    return nullptr;
  }
  const char* get_text() const { return has_text ? text.c_str() : nullptr; }
};

struct XDoc {
  std::vector<std::unique_ptr<XNode>> pool;
  XNode* root = nullptr;  // document node
  std::string err;

  XNode* make() {
    pool.emplace_back(new XNode());
    return pool.back().get();
  }

  static std::string decode(const std::string& s) {
    if (s.find('&') == std::string::npos) return s;
    std::string o;
    for (size_t i = 0; i < s.size(); ++i) {
      if (s[i] == '&') {
        size_t e = s.find(';', i);
        if (e != std::string::npos) {
          std::string ent = s.substr(i + 1, e - i - 1);
          const char* rep = nullptr;
          if (ent == "lt") rep = "<";
          else if (ent == "gt") rep = ">";
          else if (ent == "amp") rep = "&";
          else if (ent == "quot") rep = "\"";
          else if (ent == "apos") rep = "'";
          if (rep) {
            o += rep;
            i = e;
            continue;
          }
          if (!ent.empty() && ent[0] == '#') {
            long cp = ent[1] == 'x' ? std::strtol(ent.c_str() + 2, nullptr, 16) : std::strtol(ent.c_str() + 1, nullptr, 10);
            if (cp > 0 && cp < 128) {
              o += (char)cp;
              i = e;
              continue;
            }
          }
        }
      }
      o += s[i];
    }
    return o;
  }

  bool parse(const std::string& s) {
    root = make();
    XNode* cur = root;
    size_t i = 0, n = s.size();
    while (i < n) {
      if (s[i] != '<') {
        size_t j = s.find('<', i);
        if (j == std::string::npos) j = n;
        if (cur != root && cur->kids.empty() && !cur->has_text) {
          std::string t = s.substr(i, j - i);
          bool blank = t.find_first_not_of(" \t\r\n") == std::string::npos;
          if (!blank) {
            cur->text = decode(t);
            cur->has_text = true;
          }
        }
        i = j;
        continue;
      }
      if (s.compare(i, 4, "<!--") == 0) {
        size_t e = s.find("-->", i + 4);
        if (e == std::string::npos) return fail("unterminated comment");
        i = e + 3;
        continue;
      }
      if (s.compare(i, 2, "<?") == 0) {
        size_t e = s.find("?>", i + 2);
        if (e == std::string::npos) return fail("unterminated declaration");
        i = e + 2;
        continue;
      }
      if (s.compare(i, 9, "<![CDATA[") == 0) {
        size_t e = s.find("]]>", i + 9);
        if (e == std::string::npos) return fail("unterminated CDATA");
        if (cur != root && cur->kids.empty() && !cur->has_text) {
          cur->text = s.substr(i + 9, e - i - 9);
          cur->has_text = true;
        }
        i = e + 3;
        continue;
      }
      if (s.compare(i, 2, "<!") == 0) {
        size_t e = s.find('>', i + 2);
        if (e == std::string::npos) return fail("unterminated DOCTYPE");
        i = e + 1;
        continue;
      }
      if (s.compare(i, 2, "</") == 0) {
        size_t e = s.find('>', i + 2);
        if (e == std::string::npos) return fail("unterminated end tag");
        std::string nm = trim(s.substr(i + 2, e - i - 2));
        if (cur == root || cur->name != nm) return fail("mismatched end tag </" + nm + ">");
        cur = cur->parent;
        i = e + 1;
        continue;
      }
      // start tag
      size_t j = i + 1;
      while (j < n && !std::isspace((unsigned char)s[j]) && s[j] != '>' && s[j] != '/') ++j;
      XNode* e = make();
      e->name = s.substr(i + 1, j - i - 1);
      e->parent = cur;
      cur->kids.push_back(e);
      bool self_close = false;
      for (;;) {
        while (j < n && std::isspace((unsigned char)s[j])) ++j;
        if (j >= n) return fail("unterminated start tag");
        if (s[j] == '>') { ++j; break; }
        if (s[j] == '/' && j + 1 < n && s[j + 1] == '>') { j += 2; self_close = true; break; }
        size_t k = j;
        while (k < n && s[k] != '=' && !std::isspace((unsigned char)s[k])) ++k;
        std::string an = s.substr(j, k - j);
        while (k < n && s[k] != '=') ++k;
        ++k;
        while (k < n && std::isspace((unsigned char)s[k])) ++k;
        if (k >= n || (s[k] != '"' && s[k] != '\'')) return fail("bad attribute in <" + e->name + ">");
        char q = s[k];
        size_t ve = s.find(q, k + 1);
        if (ve == std::string::npos) return fail("unterminated attribute");
        e->attrs.push_back({an, decode(s.substr(k + 1, ve - k - 1))});
        j = ve + 1;
      }
      if (!self_close) cur = e;
      i = j;
    }
    if (cur != root) return fail("unclosed element <" + cur->name + ">");
    return true;
  }
  static std::string trim(const std::string& t) {
    size_t a = t.find_first_not_of(" \t\r\n"), b = t.find_last_not_of(" \t\r\n");
    return a == std::string::npos ? std::string() : t.substr(a, b - a + 1);
  }
  bool fail(const std::string& m) {
    err = m;
    return false;
  }
};

// ------------------------------------------------------------------ scene model
struct Bsdf {
  int type = 0;
  float a[3] = {0, 0, 0}, t[3] = {0, 0, 0}, e[3] = {0, 0, 0};
  float ior = 0, rough = 0;
};
struct CameraInfo {
  V3 view_dir, up_dir;
  float hFov = 0, vFov = 0, nClip = 0, fClip = 0;
};
struct LightInfo {
  int light_type = 0;  // 0 NONE 1 AMBIENT 2 DIRECTIONAL 3 AREA 4 POINT 5 SPOT
  float spectrum[3] = {1, 1, 1};
  V3 position = V3(0, 0, 0), direction = V3(0, 0, -1), up = V3(0, 1, 0);
};
struct PolymeshInfo {
  std::vector<V3> vertices;
  std::vector<std::vector<size_t>> polygons;
  int bsdf = -1;
};
struct SphereInfo {
  float radius = 0;
  int bsdf = -1;
};
enum InstType { I_NONE, I_CAMERA, I_LIGHT, I_SPHERE, I_POLYMESH };
struct Node {
  InstType type = I_NONE;
  int idx = -1;
  M4 transform = M4::identity();
};

struct Parsed {
  std::vector<Node> nodes;
  std::vector<CameraInfo> cams;
  std::vector<LightInfo> lights;
  std::vector<SphereInfo> spheres;
  std::vector<PolymeshInfo> meshes;
  std::vector<Bsdf> bsdfs;
};

struct Collada {
  XDoc doc;
  std::map<std::string, XNode*> sources;
  V3 up;
  M4 transform;  // static in the reference: zero until an <asset> sets it
  Parsed* out = nullptr;
  std::string err;

  void uri_load(XNode* x) {
    if (const char* id = x->attr("id")) sources[id] = x;
    for (XNode* c : x->kids) uri_load(c);
  }
  XNode* uri_find(const std::string& id) {
    auto it = sources.find(id);
    return it == sources.end() ? nullptr : it->second;
  }
  XNode* get_element(XNode* x, const std::string& query) {
    std::stringstream ss(query);
    XNode* e = x;
    std::string tok;
    while (e && std::getline(ss, tok, '/')) e = e->first(tok);
    if (e) {
      if (const char* url = e->attr("url")) e = uri_find(std::string(url + 1));
    }
    return e;
  }
  XNode* technique_common(XNode* x) {
    if (XNode* cp = x->first("profile_COMMON")) {
      for (XNode* t = cp->first("technique"); t; t = t->next_sibling("technique")) {
        const char* sid = t->attr("sid");
        if (sid && std::string(sid) == "common") return t;
      }
    }
    return x->first("technique_common");
  }
  XNode* technique_cmu462(XNode* x) {
    for (XNode* t = get_element(x, "extra/technique"); t; t = t->next_sibling("technique")) {
      const char* p = t->attr("profile");
      if (p && std::string(p) == "CMU462") return t;
    }
    return nullptr;
  }
  static void spectrum(const char* s, float* out) {
    std::stringstream ss(s ? s : "");
    ss >> out[0];
    ss >> out[1];
    ss >> out[2];
  }
  bool fail(const std::string& m) {
    if (err.empty()) err = m;
    return false;
  }

  bool load(const std::string& path, Parsed& P) {
    out = &P;
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return fail("cannot open " + path);
    std::string s;
    char buf[1 << 16];
    size_t k;
    while ((k = std::fread(buf, 1, sizeof(buf), f)) > 0) s.append(buf, k);
    std::fclose(f);
    if (!doc.parse(s)) return fail("XML error: " + doc.err);
    XNode* root = doc.root->first("COLLADA");
    if (!root) return fail("not a COLLADA file");
    uri_load(root);
    if (XNode* asset = get_element(root, "asset")) {
      XNode* upx = get_element(asset, "up_axis");
      if (!upx || !upx->get_text()) return fail("no up direction defined in COLLADA file");
      std::string up_dir = XDoc::trim(upx->get_text());
      transform = M4::identity();
      if (up_dir == "X_UP") {
        transform.at(0, 0) = 0; transform.at(0, 1) = 1;
        transform.at(1, 0) = 1; transform.at(1, 1) = 0;
        transform.at(2, 2) = -1;
        up = V3(1, 0, 0);
      } else if (up_dir == "Z_UP") {
        transform.at(1, 1) = 0; transform.at(1, 2) = 1;
        transform.at(2, 1) = 1; transform.at(2, 2) = 0;
        transform.at(0, 0) = -1;
        up = V3(0, 0, 1);
      } else if (up_dir == "Y_UP") {
        up = V3(0, 1, 0);
      } else {
        return fail("invalid up direction in COLLADA file");
      }
    }
    XNode* scene = get_element(root, "scene/instance_visual_scene");
    if (!scene) return fail("no scene description found");
    for (XNode* n = scene->first("node"); n; n = n->next_sibling("node"))
      if (!parse_node(n)) return false;
    return true;
  }

  bool parse_node(XNode* xml) {
    Node node;
    for (XNode* e : xml->kids) {
      const std::string& name = e->name;
      if (name == "matrix") {
        std::stringstream ss(e->get_text() ? e->get_text() : "");
        M4 mat;
        for (int i = 0; i < 4; ++i)
          for (int j = 0; j < 4; ++j) ss >> mat.at(i, j);
        node.transform = mat;
        break;
      }
      if (name == "rotate") {
        M4 m;  // zero-initialised as in the reference
        std::stringstream ss(e->get_text() ? e->get_text() : "");
        const char* sid = e->attr("sid");
        char axis = (sid && *sid) ? sid[std::strlen(sid) - 1] : 0;
        if (axis == 'X') { ss >> m.at(1, 1); ss >> m.at(1, 2); ss >> m.at(2, 1); ss >> m.at(2, 2); }
        else if (axis == 'Y') { ss >> m.at(0, 0); ss >> m.at(2, 0); ss >> m.at(0, 2); ss >> m.at(2, 2); }
        else if (axis == 'Z') { ss >> m.at(0, 0); ss >> m.at(0, 1); ss >> m.at(1, 0); ss >> m.at(1, 1); }
        node.transform = m * node.transform;
      }
      if (name == "translate") {
        M4 m;
        std::stringstream ss(e->get_text() ? e->get_text() : "");
        ss >> m.at(0, 3); ss >> m.at(1, 3); ss >> m.at(2, 3);
        node.transform = m * node.transform;
      }
      if (name == "scale") {
        M4 m;
        std::stringstream ss(e->get_text() ? e->get_text() : "");
        ss >> m.at(0, 0); ss >> m.at(1, 1); ss >> m.at(1, 1);
        node.transform = m * node.transform;
      }
    }
    M4 save = transform;
    node.transform = transform * node.transform;
    transform = node.transform;
    for (XNode* c = get_element(xml, "node"); c; c = c->next_sibling("node"))
      if (!parse_node(c)) return false;
    transform = save;

    XNode* e_camera = get_element(xml, "instance_camera");
    XNode* e_light = get_element(xml, "instance_light");
    XNode* e_geometry = get_element(xml, "instance_geometry");
    if (e_camera) {
      CameraInfo c;
      if (!parse_camera(e_camera, c)) return false;
      node.type = I_CAMERA;
      node.idx = (int)out->cams.size();
      out->cams.push_back(c);
    } else if (e_light) {
      LightInfo l;
      if (!parse_light(e_light, l)) return false;
      node.type = I_LIGHT;
      node.idx = (int)out->lights.size();
      out->lights.push_back(l);
    } else if (e_geometry) {
      if (get_element(e_geometry, "mesh")) {
        PolymeshInfo pm;
        if (!parse_polymesh(e_geometry, pm)) return false;
        pm.bsdf = instance_material(xml);
        if (pm.bsdf == -2) return false;
        node.type = I_POLYMESH;
        node.idx = (int)out->meshes.size();
        out->meshes.push_back(std::move(pm));
      } else if (get_element(e_geometry, "extra")) {
        SphereInfo sp;
        XNode* tech = technique_cmu462(e_geometry);
        if (!tech) return fail("no 462 profile technique in geometry");
        XNode* r = get_element(tech, "sphere/radius");
        if (!r || !r->get_text()) return fail("invalid sphere definition");
        sp.radius = (float)std::atof(r->get_text());
        sp.bsdf = instance_material(xml);
        if (sp.bsdf == -2) return false;
        node.type = I_SPHERE;
        node.idx = (int)out->spheres.size();
        out->spheres.push_back(sp);
      }
    }
    out->nodes.push_back(node);
    return true;
  }

  // returns bsdf index, -1 if no instance_material, -2 on error
  int instance_material(XNode* xml) {
    XNode* im = get_element(xml, "instance_geometry/bind_material/technique_common/instance_material");
    if (!im) return -1;
    const char* target = im->attr("target");
    if (!target) { fail("no target material in instance"); return -2; }
    XNode* mat = uri_find(std::string(target + 1));
    if (!mat) { fail(std::string("invalid target material id: ") + (target + 1)); return -2; }
    Bsdf b;
    if (!parse_material(mat, b)) return -2;
    out->bsdfs.push_back(b);
    return (int)out->bsdfs.size() - 1;
  }

  bool parse_camera(XNode* xml, CameraInfo& c) {
    c.up_dir = up;
    c.view_dir = V3(0, 0, -1);
    XNode* p = get_element(xml, "optics/technique_common/perspective");
    if (!p) return fail("no perspective defined in camera");
    XNode* ex = p->first("xfov");
    XNode* ey = p->first("yfov");
    XNode* en = p->first("znear");
    XNode* ef = p->first("zfar");
    c.hFov = ex ? (float)std::atof(ex->get_text() ? ex->get_text() : "") : 50.0f;
    c.vFov = ey ? (float)std::atof(ey->get_text() ? ey->get_text() : "") : 35.0f;
    c.nClip = en ? (float)std::atof(en->get_text() ? en->get_text() : "") : 0.001f;
    c.fClip = ef ? (float)std::atof(ef->get_text() ? ef->get_text() : "") : 1000.0f;
    if (!ey) {
      XNode* ar = get_element(p, "aspect_ratio");
      if (!ar) return fail("incomplete perspective definition");
      float aspect_ratio = (float)std::atof(ar->get_text() ? ar->get_text() : "");
      c.vFov = (float)(2 * degrees(std::atan(std::tan(radians(0.5 * c.hFov)) / aspect_ratio)));
    }
    return true;
  }

  bool parse_light(XNode* xml, LightInfo& l) {
    XNode* common = technique_common(xml);
    XNode* cmu = technique_cmu462(xml);
    XNode* tech = cmu ? cmu : common;
    if (!tech) return fail("no supported profile defined in light");
    XNode* e = tech->first("");
    if (!e) return true;
    const std::string& type = e->name;
    XNode* col = get_element(e, "color");
    if (type == "ambient") l.light_type = 1;
    else if (type == "directional") l.light_type = 2;
    else if (type == "area") l.light_type = 3;
    else if (type == "point") l.light_type = 4;
    else if (type == "spot") l.light_type = 5;
    else return fail("light type " + type + " is not supported");
    if (!col || !col->get_text()) return fail("no color definition in light");
    spectrum(col->get_text(), l.spectrum);
    return true;
  }

  bool parse_polymesh(XNode* xml, PolymeshInfo& pm) {
    XNode* mesh = xml->first("mesh");
    if (!mesh) return fail("no mesh data defined in geometry");
    std::map<std::string, std::vector<float>> arr;
    for (XNode* src = mesh->first("source"); src; src = src->next_sibling("source")) {
      XNode* fa = src->first("float_array");
      if (!fa) continue;
      const char* sid = src->attr("id");
      const char* cnt = fa->attr("count");
      size_t n = cnt ? (size_t)std::atoi(cnt) : 0;
      std::vector<float> v;
      v.reserve(n);
      const char* p = fa->get_text() ? fa->get_text() : "";
      char* endp = nullptr;
      float last = 0.f;
      for (size_t i = 0; i < n; ++i) {
        float f = std::strtof(p, &endp);
        if (endp == p) f = last;  // stream failure keeps the previous value
        else p = endp;
        last = f;
        v.push_back(f);
      }
      arr[sid ? sid : ""] = std::move(v);
    }
    XNode* verts = mesh->first("vertices");
    if (!verts) return fail("no vertices defined in geometry");
    std::string vid = verts->attr("id") ? verts->attr("id") : "";
    std::vector<V3> vertices;
    for (XNode* in = verts->first("input"); in; in = in->next_sibling("input")) {
      const char* sem = in->attr("semantic");
      if (sem && std::string(sem) == "POSITION") {
        std::string s = in->attr("source") ? in->attr("source") + 1 : "";
        auto it = arr.find(s);
        if (it == arr.end()) return fail("undefined input source: " + s);
        const std::vector<float>& fl = it->second;
        for (size_t i = 0; i + 2 < fl.size() + 0 && i < fl.size(); i += 3)
          vertices.push_back(V3(fl[i], fl[i + 1], fl[i + 2]));
      }
    }
    XNode* pl = mesh->first("polylist");
    if (!pl) return true;
    bool has_v = false, has_n = false, has_t = false;
    size_t voff = 0;
    for (XNode* in = pl->first("input"); in; in = in->next_sibling("input")) {
      std::string sem = in->attr("semantic") ? in->attr("semantic") : "";
      std::string src = in->attr("source") ? in->attr("source") + 1 : "";
      size_t off = in->attr("offset") ? (size_t)std::atoi(in->attr("offset")) : 0;
      if (sem == "VERTEX") {
        has_v = true;
        voff = off;
        if (src != vid) return fail("undefined source for VERTEX semantic: " + src);
        pm.vertices = vertices;
      }
      if (sem == "NORMAL") {
        has_n = true;
        if (!arr.count(src)) return fail("undefined source for NORMAL semantic: " + src);
      }
      if (sem == "TEXCOORD") {
        has_t = true;
        if (!arr.count(src)) return fail("undefined source for TEXCOORD semantic: " + src);
      }
    }
    const char* cnt = pl->attr("count");
    size_t npoly = cnt ? (size_t)std::atoi(cnt) : 0;
    size_t stride = (has_v ? 1 : 0) + (has_n ? 1 : 0) + (has_t ? 1 : 0);
    XNode* vc = pl->first("vcount");
    if (!vc) return fail("polygon sizes undefined in geometry");
    std::vector<size_t> sizes;
    size_t nidx = 0;
    {
      const char* p = vc->get_text() ? vc->get_text() : "";
      char* endp;
      for (size_t i = 0; i < npoly; ++i) {
        size_t v = (size_t)std::strtoull(p, &endp, 10);
        p = endp;
        sizes.push_back(v);
        nidx += v * stride;
      }
    }
    XNode* pe = pl->first("p");
    if (!pe) return fail("no index array defined in geometry");
    std::vector<size_t> idx;
    idx.reserve(nidx);
    {
      const char* p = pe->get_text() ? pe->get_text() : "";
      char* endp;
      for (size_t i = 0; i < nidx; ++i) {
        size_t v = (size_t)std::strtoull(p, &endp, 10);
        p = endp;
        idx.push_back(v);
      }
    }
    pm.polygons.resize(npoly);
    if (has_v) {
      size_t k = 0;
      for (size_t i = 0; i < npoly; ++i)
        for (size_t j = 0; j < sizes[i]; ++j) {
          pm.polygons[i].push_back(idx[k * stride + voff]);
          k++;
        }
    }
    return true;
  }

  bool parse_material(XNode* xml, Bsdf& b) {
    XNode* eff = get_element(xml, "instance_effect");
    if (!eff) return fail("no target effects found for material");
    XNode* common = technique_common(eff);
    XNode* cmu = technique_cmu462(eff);
    if (cmu) {
      for (XNode* e : cmu->kids) {
        const std::string& type = e->name;
        auto txt = [&](const char* q) -> const char* {
          XNode* x = get_element(e, q);
          return x ? x->get_text() : nullptr;
        };
        if (type == "emission") {
          b = Bsdf();
          b.type = 4;
          spectrum(txt("radiance"), b.e);
        } else if (type == "mirror") {
          b = Bsdf();
          b.type = 1;
          spectrum(txt("reflectance"), b.a);
        } else if (type == "refraction") {
          b = Bsdf();
          b.type = 2;
          spectrum(txt("transmittance"), b.t);
          b.rough = (float)std::atof(txt("roughness") ? txt("roughness") : "");
          b.ior = (float)std::atof(txt("ior") ? txt("ior") : "");
        } else if (type == "glass") {
          b = Bsdf();
          b.type = 3;
          spectrum(txt("transmittance"), b.t);
          spectrum(txt("reflectance"), b.a);
          b.rough = (float)std::atof(txt("roughness") ? txt("roughness") : "");
          b.ior = (float)std::atof(txt("ior") ? txt("ior") : "");
        }
      }
    } else if (common) {
      XNode* d = get_element(common, "phong/diffuse/color");
      b = Bsdf();
      b.type = 0;
      if (d) spectrum(d->get_text(), b.a);
      else b.a[0] = b.a[1] = b.a[2] = .5f;
    } else {
      b = Bsdf();
      b.type = 0;
      b.a[0] = b.a[1] = b.a[2] = .5f;
    }
    return true;
  }
};

// ------------------------------------------------------------------ halfedge
// Index-based restatement of HalfedgeMesh::build: same creation order of
// vertices (first appearance), halfedges (face order, then boundary loops),
// twin/next links and vertex->halfedge choice, so Vertex::computeNormal sums
// its cross products in the reference's order.
struct HalfedgeMesh {
  struct H { int next = -1, twin = -1, vertex = -1, face = -1; bool boundary_face = false; };
  std::vector<H> he;
  std::vector<int> v_he;        // vertex -> halfedge
  std::vector<V3> v_pos, v_nrm;
  std::vector<int> f_he;        // face -> halfedge
  std::vector<size_t> v_index;  // vertex -> source index

  bool build(const std::vector<std::vector<size_t>>& polygons, const std::vector<V3>& positions, std::string& err) {
    std::map<size_t, int> indexToVertex;
    std::vector<size_t> degree;
    for (const auto& p : polygons) {
      if (p.size() < 3) { err = "polygon with fewer than three vertices"; return false; }
      std::set<size_t> uniq;
      for (size_t i : p) {
        uniq.insert(i);
        auto it = indexToVertex.find(i);
        if (it == indexToVertex.end()) {
          int v = (int)v_he.size();
          v_he.push_back(-1);
          v_index.push_back(i);
          indexToVertex[i] = v;
          degree.push_back(1);
        } else {
          degree[it->second]++;
        }
      }
      if (uniq.size() < p.size()) { err = "polygon without distinct vertices"; return false; }
    }
    f_he.assign(polygons.size(), -1);
    std::map<std::pair<size_t, size_t>, int> pairToHalfedge;
    for (size_t f = 0; f < polygons.size(); ++f) {
      const auto& p = polygons[f];
      size_t deg = p.size();
      std::vector<int> fh;
      for (size_t i = 0; i < deg; ++i) {
        size_t a = p[i], b = p[(i + 1) % deg];
        if (pairToHalfedge.count({a, b})) { err = "non-manifold or inconsistently oriented mesh"; return false; }
        int hab = (int)he.size();
        he.push_back(H());
        pairToHalfedge[{a, b}] = hab;
        he[hab].face = (int)f;
        f_he[f] = hab;
        he[hab].vertex = indexToVertex[a];
        v_he[he[hab].vertex] = hab;
        fh.push_back(hab);
        auto iba = pairToHalfedge.find({b, a});
        if (iba != pairToHalfedge.end()) {
          he[hab].twin = iba->second;
          he[iba->second].twin = hab;
        } else {
          he[hab].twin = -1;
        }
      }
      for (size_t i = 0; i < deg; ++i) he[fh[i]].next = fh[(i + 1) % deg];
    }
    // advance boundary vertices to a halfedge without twin
    for (size_t v = 0; v < v_he.size(); ++v) {
      int h = v_he[v];
      int start = h;
      do {
        if (he[h].twin < 0) {
          v_he[v] = h;
          break;
        }
        h = he[he[h].twin].next;
      } while (h != start);
    }
    // boundary loops (the list grows while it is walked; new ones have twins)
    for (size_t hi = 0; hi < he.size(); ++hi) {
      if (he[hi].twin >= 0) continue;
      std::vector<int> bh;
      int h = (int)hi, i = h;
      do {
        int t = (int)he.size();
        he.push_back(H());
        he[t].boundary_face = true;
        bh.push_back(t);
        he[i].twin = t;
        he[t].twin = i;
        he[t].vertex = he[he[i].next].vertex;
        i = he[i].next;
        while (i != h && he[i].twin >= 0) {
          i = he[i].twin;
          i = he[i].next;
        }
      } while (i != h);
      size_t deg = bh.size();
      for (size_t p = 0; p < deg; ++p) he[bh[p]].next = bh[(p - 1 + deg) % deg];
    }
    for (size_t v = 0; v < v_he.size(); ++v) v_he[v] = he[he[v_he[v]].twin].next;
    for (size_t v = 0; v < v_he.size(); ++v) {
      size_t count = 0;
      int h = v_he[v];
      do {
        if (!he[h].boundary_face) count++;
        h = he[he[h].twin].next;
      } while (h != v_he[v]);
      if (count != degree[v]) { err = "non-manifold vertex"; return false; }
    }
    if (positions.size() != v_he.size()) { err = "vertex positions / referenced vertices mismatch"; return false; }
    v_pos.resize(v_he.size());
    {
      int i = 0;
      for (auto& kv : indexToVertex) v_pos[kv.second] = positions[i++];
    }
    v_nrm.resize(v_he.size());
    for (size_t v = 0; v < v_he.size(); ++v) v_nrm[v] = compute_normal((int)v);
    return true;
  }

  bool vertex_is_boundary(int v) const {
    int h = v_he[v];
    do {
      if (he[h].boundary_face) return true;
      h = he[he[h].twin].next;
    } while (h != v_he[v]);
    return false;
  }

  V3 compute_normal(int v) const {
    V3 n(0., 0., 0.);
    V3 pi = v_pos[v];
    int h = v_he[v];
    if (vertex_is_boundary(v)) {
      do {
        V3 pj = v_pos[he[he[h].next].vertex];
        V3 pk = v_pos[he[he[he[h].next].next].vertex];
        n += cross(pj - pi, pk - pi);
        h = he[he[h].next].twin;
      } while (h != v_he[v]);
    } else {
      do {
        V3 pj = v_pos[he[he[h].next].vertex];
        V3 pk = v_pos[he[he[he[h].next].next].vertex];
        n += cross(pj - pi, pk - pi);
        h = he[he[h].twin].next;
      } while (h != v_he[v]);
    }
    n.normalize();
    return n;
  }
};

// ------------------------------------------------------------------ static scene
struct Prim {
  int type;  // 0 sphere, 1 triangle
  int bsdf;
  int orig;
  V3 p[3], n[3];
  double r = 0;
  BBox bbox() const {
    if (type == 0) return BBox(p[0] - V3(r, r, r), p[0] + V3(r, r, r));
    BBox b;
    b.expand(p[0]);
    b.expand(p[1]);
    b.expand(p[2]);
    return b;
  }
};

struct BNode {
  BBox bb;
  int64_t start, range;
  int l = -1, r = -1;
};

struct BvhBuilder {
  std::vector<Prim>& prims;
  std::vector<BNode> nodes;
  std::vector<BBox> pbb;  // bbox per primitive slot (permuted with prims)
  explicit BvhBuilder(std::vector<Prim>& p) : prims(p) {}

  struct Bucket {
    BBox bb;
    int prim_count = 0;
  };

  void swap_prim(int i, int j) {
    std::swap(prims[i], prims[j]);
    std::swap(pbb[i], pbb[j]);
  }

  // buildBVH (bvh.cpp:21-178)
  void build(int ni, int bucketNum, size_t max_leaf) {
    BBox lbb, rbb;
    int lRange, rRange;
    {
      double minC[3] = {INF_D, INF_D, INF_D};
      int minBIndex[3] = {0, 0, 0};
      const BNode node = nodes[ni];
      for (int k = 0; k < 3; k++) {
        double ub = node.bb.max[k];
        double lb = node.bb.min[k];
        if (ub == lb) continue;
        double interval = (ub - lb) / bucketNum;
        std::vector<Bucket> B(bucketNum), rB(bucketNum);
        for (int i = 0; i < node.range; i++) {
          const BBox& b = pbb[node.start + i];
          double c = (b.min[k] + b.max[k]) * 0.5;
          int bIndex = (c - lb) / interval;
          if (bIndex >= bucketNum) bIndex = bucketNum - 1;
          B[bIndex].bb.expand(b);
          B[bIndex].prim_count++;
        }
        for (int i = 0; i < bucketNum; i++) {
          rB[i] = B[bucketNum - i - 1];
          if (i > 0) {
            rB[i].bb.expand(rB[i - 1].bb);
            rB[i].prim_count += rB[i - 1].prim_count;
          }
        }
        for (int i = 1; i < bucketNum; i++) {
          B[i].bb.expand(B[i - 1].bb);
          B[i].prim_count += B[i - 1].prim_count;
        }
        for (int i = 0; i < bucketNum - 1; i++) {
          Bucket& b1 = B[i];
          Bucket& b2 = rB[bucketNum - i - 2];
          double C = (b1.bb.extent.x * b1.bb.extent.y + b1.bb.extent.x * b1.bb.extent.z +
                      b1.bb.extent.y * b1.bb.extent.z) * b1.prim_count +
                     (b2.bb.extent.x * b2.bb.extent.y + b2.bb.extent.x * b2.bb.extent.z +
                      b2.bb.extent.y * b2.bb.extent.z) * b2.prim_count;
          if (C < minC[k]) {
            minC[k] = C;
            minBIndex[k] = i + 1;
          }
        }
      }
      int axis = 0;
      double cost = minC[0];
      for (int i = 1; i < 3; i++)
        if (minC[i] < cost) {
          axis = i;
          cost = minC[i];
        }
      double ub = node.bb.max[axis];
      double lb = node.bb.min[axis];
      double pLine = lb + (ub - lb) * minBIndex[axis] / bucketNum;
      int i = (int)node.start - 1;
      int j = (int)(node.start + node.range);
      BBox bb1, bb2;
      while (i < j) {
        do {
          i++;
          if (i >= (int)(node.start + node.range)) break;
          bb1 = pbb[i];
        } while ((bb1.min[axis] + bb1.max[axis]) * 0.5 < pLine);
        do {
          j--;
          if (j < (int)node.start) break;
          bb2 = pbb[j];
        } while ((bb2.min[axis] + bb2.max[axis]) * 0.5 > pLine);
        if (i < j) swap_prim(i, j);
        else break;
      }
      lRange = i - (int)node.start;
      rRange = (int)node.range - lRange;
      for (int jj = 0; jj < node.range; jj++) {
        bb1 = pbb[node.start + jj];
        if (jj < lRange) lbb.expand(bb1);
        else rbb.expand(bb1);
      }
    }
    int start = (int)nodes[ni].start;
    if (!(lRange == 0 || rRange == 0)) {
      BNode L, R;
      L.bb = lbb;
      L.start = start;
      L.range = lRange;
      R.bb = rbb;
      R.start = start + lRange;
      R.range = rRange;
      int li = (int)nodes.size();
      nodes.push_back(L);
      int ri = (int)nodes.size();
      nodes.push_back(R);
      nodes[ni].l = li;
      nodes[ni].r = ri;
    }
    if ((size_t)lRange <= max_leaf && (size_t)rRange <= max_leaf) return;
    if ((size_t)lRange <= max_leaf) {
      if (lRange > 0) build(nodes[ni].r, bucketNum, max_leaf);
    } else if ((size_t)rRange <= max_leaf) {
      if (rRange > 0) build(nodes[ni].l, bucketNum, max_leaf);
    } else {
      int l = nodes[ni].l, r = nodes[ni].r;
      build(l, bucketNum, max_leaf);
      build(r, bucketNum, max_leaf);
    }
  }

  void run() {
    pbb.resize(prims.size());
    BBox bb;
    for (size_t i = 0; i < prims.size(); ++i) {
      pbb[i] = prims[i].bbox();
      bb.expand(pbb[i]);
    }
    BNode root;
    root.bb = bb;
    root.start = 0;
    root.range = (int64_t)prims.size();
    nodes.push_back(root);
    build(0, 32, 4);
  }
};

struct Camera {
  double hFov = 0, vFov = 0, ar = 0, nClip = 0, fClip = 0;
  V3 pos, targetPos;
  double phi = 0, theta = 0, r = 0, minR = 0, maxR = 0;
  V3 c2w[3];  // columns
  size_t screenW = 0, screenH = 0;
  double screenDist = 0;

  void configure(const CameraInfo& info, size_t W, size_t H) {
    screenW = W;
    screenH = H;
    nClip = info.nClip;
    fClip = info.fClip;
    hFov = info.hFov;
    vFov = info.vFov;
    double ar1 = std::tan(radians(hFov) / 2) / std::tan(radians(vFov) / 2);
    ar = static_cast<double>(W) / H;
    if (ar1 < ar) hFov = 2 * degrees(std::atan(std::tan(radians(vFov) / 2) * ar));
    else if (ar1 > ar) vFov = 2 * degrees(std::atan(std::tan(radians(hFov) / 2) / ar));
    screenDist = ((double)H) / (2.0 * std::tan(radians(vFov) / 2));
  }
  void place(const V3& target, double ph, double th, double rr, double mn, double mx) {
    double r_ = std::min(std::max(rr, mn), mx);
    double phi_ = (std::sin(ph) == 0) ? (ph + EPS_F) : ph;
    targetPos = target;
    phi = phi_;
    theta = th;
    r = r_;
    minR = mn;
    maxR = mx;
    compute_position();
  }
  void compute_position() {
    double sinPhi = std::sin(phi);
    if (sinPhi == 0) {
      phi += EPS_F;
      sinPhi = std::sin(phi);
    }
    const V3 dirToCamera(r * sinPhi * std::sin(theta), r * std::cos(phi), r * sinPhi * std::cos(theta));
    pos = targetPos + dirToCamera;
    V3 upVec(0, sinPhi > 0 ? 1 : -1, 0);
    V3 sx = cross(upVec, dirToCamera);
    sx.normalize();
    V3 sy = cross(dirToCamera, sx);
    sy.normalize();
    c2w[0] = sx;
    c2w[1] = sy;
    c2w[2] = dirToCamera.unit();
  }
};

}  // namespace hs

// ------------------------------------------------------------------ C ABI object
struct pt_host_scene {
  std::vector<int32_t> prim_type, prim_bsdf, prim_orig;
  std::vector<double> prim_geom, prim_norm;
  std::vector<pt_bvh_node> nodes;
  std::vector<pt_bsdf> bsdfs;
  std::vector<pt_light> lights;
  pt_camera cam{};
  double hfov = 0, vfov = 0;
  int32_t env_w = 0, env_h = 0;  // EnvironmentLight map (pt_host_scene_set_envmap)
  std::vector<float> env_rgb;
};

namespace {

int load_impl(const char* path, int W, int H, const char* cam_info, pt_host_scene* out) {
  using namespace hs;
  Collada col;
  Parsed P;
  if (!col.load(path, P)) return pt_fail(PT_E_INVALID, "pt_host_scene_load: " + col.err);

  // Application::load (application.cpp:223-299)
  Camera camera;
  bool have_cam = false;
  V3 c_pos, c_dir;
  struct DynLight { int type; float rad[3]; V3 position, direction, dim_x, dim_y; };
  std::vector<DynLight> lights;
  struct Obj { int kind; int idx; M4 tr; V3 sp_pos; double sp_r; };
  std::vector<Obj> objects;
  for (const Node& node : P.nodes) {
    const M4& T = node.transform;
    switch (node.type) {
      case I_CAMERA: {
        const CameraInfo& c = P.cams[node.idx];
        c_pos = (T * V4(c_pos, 1)).to3D();
        c_dir = (T * V4(c.view_dir, 1)).to3D().unit();
        camera.configure(c, (size_t)W, (size_t)H);
        have_cam = true;
        break;
      }
      case I_LIGHT: {
        const LightInfo& li = P.lights[node.idx];
        DynLight d;
        std::memcpy(d.rad, li.spectrum, sizeof(d.rad));
        if (li.light_type == 3) {  // DynamicScene::AreaLight (area_light.h:12-25)
          d.type = PT_LIGHT_AREA;
          d.position = (T * V4(li.position, 1)).to3D();
          d.direction = (T * V4(li.direction, 1)).to3D() - d.position;
          d.direction.normalize();
          V3 dy = li.up;
          V3 dx = cross(li.up, li.direction);
          d.dim_x = (T * V4(dx, 1)).to3D() - d.position;
          d.dim_y = (T * V4(dy, 1)).to3D() - d.position;
        } else if (li.light_type == 2) {  // DirectionalLight (directional_light.h)
          d.type = PT_LIGHT_DIRECTIONAL;
          V3 dir = -(T * V4(li.direction, 1)).to3D();
          dir.normalize();
          d.direction = -dir.unit();  // StaticScene::DirectionalLight stores dirToLight
        } else if (li.light_type == 4) {  // PointLight (point_light.h)
          d.type = PT_LIGHT_POINT;
          d.position = (T * V4(li.position, 1)).to3D();
        } else if (li.light_type == 1) {  // AmbientLight -> InfiniteHemisphereLight
          d.type = PT_LIGHT_HEMISPHERE;
        } else {
          return pt_fail(PT_E_INVALID, "pt_host_scene_load: spot lights are stubs in the reference (light.cpp:61-69)");
        }
        lights.push_back(d);
        break;
      }
      case I_SPHERE: {
        Obj o;
        o.kind = 0;
        o.idx = node.idx;
        o.sp_pos = (T * V4(0, 0, 0, 1)).projectTo3D();
        double scale = (T * V4(1, 0, 0, 0)).to3D().norm();
        o.sp_r = P.spheres[node.idx].radius * scale;
        objects.push_back(o);
        break;
      }
      case I_POLYMESH: {
        Obj o;
        o.kind = 1;
        o.idx = node.idx;
        o.tr = T;
        objects.push_back(o);
        break;
      }
      default:
        break;
    }
  }
  if (!have_cam) return pt_fail(PT_E_INVALID, "pt_host_scene_load: the scene has no camera");

  // Objects -> static primitives (pathtracer.cpp:230-234), BSDF per object.
  std::vector<Prim> prims;
  std::vector<Bsdf> bsdf_table;
  BBox scene_bb;
  for (const Obj& o : objects) {
    int bsdf_src = o.kind == 0 ? P.spheres[o.idx].bsdf : P.meshes[o.idx].bsdf;
    Bsdf b;
    if (bsdf_src >= 0) b = P.bsdfs[bsdf_src];
    else { b.type = 0; b.a[0] = b.a[1] = b.a[2] = 0.5f; }
    int bi = (int)bsdf_table.size();
    bsdf_table.push_back(b);
    if (o.kind == 0) {
      Prim p;
      p.type = 0;
      p.bsdf = bi;
      p.orig = (int)prims.size();
      p.p[0] = o.sp_pos;
      p.r = o.sp_r;
      prims.push_back(p);
      scene_bb.expand(BBox(V3(o.sp_pos.x - o.sp_r, o.sp_pos.y - o.sp_r, o.sp_pos.z - o.sp_r),
                           V3(o.sp_pos.x + o.sp_r, o.sp_pos.y + o.sp_r, o.sp_pos.z + o.sp_r)));
      continue;
    }
    const PolymeshInfo& pm = P.meshes[o.idx];
    std::vector<V3> verts = pm.vertices;
    for (V3& v : verts) v = (o.tr * V4(v, 1)).projectTo3D();
    HalfedgeMesh hm;
    std::string err;
    if (!hm.build(pm.polygons, verts, err)) return pt_fail(PT_E_INVALID, "pt_host_scene_load: halfedge build: " + err);
    BBox mb;
    for (const V3& p : hm.v_pos) mb.expand(p);
    scene_bb.expand(mb);
    // StaticScene::Mesh: vertices in list order, each face's first three
    // vertices starting at its halfedge (the last one created for the face).
    for (size_t f = 0; f < hm.f_he.size(); ++f) {
      int h0 = hm.f_he[f];
      int vi[3] = {hm.he[h0].vertex, hm.he[hm.he[h0].next].vertex, hm.he[hm.he[hm.he[h0].next].next].vertex};
      Prim p;
      p.type = 1;
      p.bsdf = bi;
      p.orig = (int)prims.size();
      for (int k = 0; k < 3; ++k) {
        p.p[k] = hm.v_pos[vi[k]];
        p.n[k] = hm.v_nrm[vi[k]];
      }
      prims.push_back(p);
    }
  }
  if (prims.empty()) return pt_fail(PT_E_INVALID, "pt_host_scene_load: the scene has no primitives");

  if (!scene_bb.empty()) {
    V3 target = scene_bb.centroid();
    double canonical = scene_bb.extent.norm() / 2 * 1.5;
    double view_distance = canonical * 2;
    camera.place(target, std::acos(c_dir.y), std::atan2(c_dir.x, c_dir.z), view_distance, canonical / 10.0,
                 canonical * 20.0);
  }
  if (cam_info && *cam_info) {  // Application::loadCamera (application.cpp:823-853)
    FILE* f = std::fopen(cam_info, "r");
    if (!f) return pt_fail(PT_E_IO, std::string("pt_host_scene_load: cannot open camera file ") + cam_info);
    double m[9];
    int n = 0;
    n += std::fscanf(f, "%lf %lf %lf", &camera.pos.x, &camera.pos.y, &camera.pos.z);
    n += std::fscanf(f, "%lf %lf %lf", &camera.targetPos.x, &camera.targetPos.y, &camera.targetPos.z);
    n += std::fscanf(f, "%lf", &camera.phi);
    n += std::fscanf(f, "%lf", &camera.theta);
    n += std::fscanf(f, "%lf", &camera.minR);
    n += std::fscanf(f, "%lf", &camera.maxR);
    n += std::fscanf(f, "%lf %lf %lf %lf %lf %lf %lf %lf %lf", &m[0], &m[1], &m[2], &m[3], &m[4], &m[5], &m[6], &m[7],
                     &m[8]);
    std::fclose(f);
    if (n != 19) return pt_fail(PT_E_IO, "pt_host_scene_load: malformed camera file");
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) camera.c2w[j][i] = m[3 * i + j];
  }

  // BVH (pathtracer.cpp:242 -> bvh.cpp:181-202).  A non-finite coordinate
  // (a corrupted or hostile file: "nan", "1e999") would turn the bucket index
  // of bvh.cpp:47 into an out-of-range integer conversion; the reference reads
  // out of bounds there, this pipeline refuses the scene.
  if (prims.empty()) return pt_fail(PT_E_IO, "pt_host_scene_load: the scene has no primitives");
  for (const Prim& p : prims) {
    const BBox b = p.bbox();
    for (int k = 0; k < 3; ++k)
      if (!std::isfinite(b.min[k]) || !std::isfinite(b.max[k]))
        return pt_fail(PT_E_IO, "pt_host_scene_load: non-finite primitive coordinate");
  }
  BvhBuilder bb(prims);
  bb.run();

  // ---- flatten
  out->prim_type.resize(prims.size());
  out->prim_bsdf.resize(prims.size());
  out->prim_orig.resize(prims.size());
  out->prim_geom.assign(prims.size() * 9, 0.0);
  out->prim_norm.assign(prims.size() * 9, 0.0);
  for (size_t i = 0; i < prims.size(); ++i) {
    const Prim& p = prims[i];
    out->prim_type[i] = p.type;
    out->prim_bsdf[i] = p.bsdf;
    out->prim_orig[i] = p.orig;
    double* g = &out->prim_geom[9 * i];
    double* n = &out->prim_norm[9 * i];
    if (p.type == 1) {
      for (int k = 0; k < 3; ++k) {
        g[3 * k] = p.p[k].x; g[3 * k + 1] = p.p[k].y; g[3 * k + 2] = p.p[k].z;
        n[3 * k] = p.n[k].x; n[3 * k + 1] = p.n[k].y; n[3 * k + 2] = p.n[k].z;
      }
    } else {
      g[0] = p.p[0].x; g[1] = p.p[0].y; g[2] = p.p[0].z; g[3] = p.r;
    }
  }
  // nodes in pre-order (node, left subtree, right subtree)
  std::vector<int> order, id(bb.nodes.size(), -1);
  std::vector<int> st = {0};
  while (!st.empty()) {
    int n = st.back();
    st.pop_back();
    id[n] = (int)order.size();
    order.push_back(n);
    if (bb.nodes[n].r >= 0) st.push_back(bb.nodes[n].r);
    if (bb.nodes[n].l >= 0) st.push_back(bb.nodes[n].l);
  }
  out->nodes.resize(order.size());
  for (size_t i = 0; i < order.size(); ++i) {
    const BNode& N = bb.nodes[order[i]];
    pt_bvh_node& o = out->nodes[i];
    for (int k = 0; k < 3; ++k) {
      o.bb_min[k] = N.bb.min[k];
      o.bb_max[k] = N.bb.max[k];
    }
    o.start = N.start;
    o.range = N.range;
    o.left = N.l >= 0 ? id[N.l] : -1;
    o.right = N.r >= 0 ? id[N.r] : -1;
  }
  out->bsdfs.resize(bsdf_table.size());
  for (size_t i = 0; i < bsdf_table.size(); ++i) {
    const Bsdf& b = bsdf_table[i];
    pt_bsdf& o = out->bsdfs[i];
    o.type = b.type;
    for (int k = 0; k < 3; ++k) {
      o.albedo[k] = b.a[k];
      o.transmittance[k] = b.t[k];
      o.emission[k] = b.e[k];
    }
    o.ior = b.ior;
    o.roughness = b.rough;
  }
  out->lights.resize(lights.size());
  for (size_t i = 0; i < lights.size(); ++i) {
    const DynLight& d = lights[i];
    pt_light& o = out->lights[i];
    std::memset(&o, 0, sizeof(o));
    o.type = d.type;
    for (int k = 0; k < 3; ++k) {
      o.radiance[k] = d.rad[k];
      o.position[k] = d.position[k];
      o.direction[k] = d.direction[k];
      o.dim_x[k] = d.dim_x[k];
      o.dim_y[k] = d.dim_y[k];
    }
    // AreaLight::area = |dim_x| * |dim_y| in float (light.cpp:74-78)
    o.area = d.type == PT_LIGHT_AREA ? (float)(d.dim_x.norm() * d.dim_y.norm()) : 0.f;
  }
  for (int k = 0; k < 3; ++k) out->cam.pos[k] = camera.pos[k];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) out->cam.c2w[3 * i + j] = camera.c2w[j][i];
  out->cam.screen_w = (double)camera.screenW;
  out->cam.screen_h = (double)camera.screenH;
  out->cam.screen_dist = camera.screenDist;
  out->hfov = camera.hFov;
  out->vfov = camera.vFov;
  return PT_OK;
}

}  // namespace

extern "C" {

int pt_host_scene_load(const char* dae_path, int32_t width, int32_t height, const char* cam_info,
                       pt_host_scene** out) {
  if (!dae_path || !out) return pt_fail(PT_E_INVALID, "pt_host_scene_load: NULL argument");
  *out = nullptr;
  if (width <= 0 || height <= 0) return pt_fail(PT_E_INVALID, "pt_host_scene_load: non-positive frame size");
  pt_host_scene* s = new pt_host_scene();
  int rc;
  try {
    rc = load_impl(dae_path, width, height, cam_info, s);
  } catch (const std::bad_alloc&) {
    rc = pt_fail(PT_E_ALLOC, "pt_host_scene_load: out of memory");
  } catch (const std::exception& e) {
    rc = pt_fail(PT_E_INVALID, std::string("pt_host_scene_load: ") + e.what());
  }
  if (rc != PT_OK) {
    delete s;
    return rc;
  }
  *out = s;
  return PT_OK;
}

int pt_host_scene_view(const pt_host_scene* s, pt_scene* scene, pt_camera* cam) {
  if (!s) return pt_fail(PT_E_INVALID, "pt_host_scene_view: NULL scene");
  if (scene) {
    scene->n_prims = (int64_t)s->prim_type.size();
    scene->prim_type = s->prim_type.data();
    scene->prim_bsdf = s->prim_bsdf.data();
    scene->prim_geom = s->prim_geom.data();
    scene->prim_norm = s->prim_norm.data();
    scene->n_nodes = (int64_t)s->nodes.size();
    scene->nodes = s->nodes.data();
    scene->n_bsdfs = (int32_t)s->bsdfs.size();
    scene->bsdfs = s->bsdfs.data();
    scene->n_lights = (int32_t)s->lights.size();
    scene->lights = s->lights.data();
    scene->env_width = s->env_w;
    scene->env_height = s->env_h;
    scene->env_rgb = s->env_w > 0 ? s->env_rgb.data() : nullptr;
  }
  if (cam) *cam = s->cam;
  return PT_OK;
}

int pt_host_scene_dump(const pt_host_scene* s, const char* path) {
  if (!s || !path) return pt_fail(PT_E_INVALID, "pt_host_scene_dump: NULL argument");
  ptdump::Writer w(path);
  if (!w.ok()) return pt_fail(PT_E_IO, std::string("pt_host_scene_dump: cannot write ") + path);
  std::vector<double> cam(s->cam.pos, s->cam.pos + 3);
  cam.insert(cam.end(), s->cam.c2w, s->cam.c2w + 9);
  cam.push_back(s->cam.screen_w);
  cam.push_back(s->cam.screen_h);
  cam.push_back(s->cam.screen_dist);
  cam.push_back(s->hfov);
  cam.push_back(s->vfov);
  w.f8("cam", cam);
  std::vector<int32_t> bt;
  std::vector<float> bp;
  for (const pt_bsdf& b : s->bsdfs) {
    bt.push_back(b.type);
    float p[12] = {b.albedo[0], b.albedo[1], b.albedo[2], b.transmittance[0], b.transmittance[1],
                   b.transmittance[2], b.emission[0], b.emission[1], b.emission[2], b.ior, b.roughness, 0.f};
    bp.insert(bp.end(), p, p + 12);
  }
  w.i4("bsdf_type", bt);
  w.f4("bsdf_params", bp);
  std::vector<int32_t> lt;
  std::vector<float> lr, la;
  std::vector<double> lg;
  for (const pt_light& l : s->lights) {
    lt.push_back(l.type);
    lr.insert(lr.end(), l.radiance, l.radiance + 3);
    lg.insert(lg.end(), l.position, l.position + 3);
    lg.insert(lg.end(), l.direction, l.direction + 3);
    lg.insert(lg.end(), l.dim_x, l.dim_x + 3);
    lg.insert(lg.end(), l.dim_y, l.dim_y + 3);
    la.push_back(l.area);
  }
  w.i4("light_type", lt);
  w.f4("light_rad", lr);
  w.f8("light_geom", lg);
  w.f4("light_area", la);
  if (s->env_w > 0) {
    w.i8("env_shape", {(int64_t)s->env_h, (int64_t)s->env_w});
    w.f4("env_rgb", s->env_rgb);
  }
  w.i4("prim_type", s->prim_type);
  w.i4("prim_bsdf", s->prim_bsdf);
  w.i4("prim_orig", s->prim_orig);
  w.f8("prim_geom", s->prim_geom);
  w.f8("prim_norm", s->prim_norm);
  std::vector<double> nbb;
  std::vector<int64_t> ni;
  for (const pt_bvh_node& n : s->nodes) {
    nbb.insert(nbb.end(), n.bb_min, n.bb_min + 3);
    nbb.insert(nbb.end(), n.bb_max, n.bb_max + 3);
    ni.push_back(n.start);
    ni.push_back(n.range);
    ni.push_back(n.left);
    ni.push_back(n.right);
  }
  w.f8("node_bb", nbb);
  w.i8("node_info", ni);
  w.close();
  return PT_OK;
}

// PathTracer(..., envmap) + set_scene (src/pathtracer.cpp:42-46, 88-90): the
// environment light joins the scene's lights last; main.cpp -e loads the map.
int pt_host_scene_set_envmap(pt_host_scene* s, const char* exr_path) {
  if (!s || !exr_path) return pt_fail(PT_E_INVALID, "pt_host_scene_set_envmap: NULL argument");
  int32_t w = 0, h = 0;
  float* rgb = nullptr;
  int rc = pt_host_load_exr(exr_path, &w, &h, &rgb);
  if (rc) return rc;
  s->env_rgb.assign(rgb, rgb + (size_t)w * h * 3);
  pt_host_free(rgb);
  s->env_w = w;
  s->env_h = h;
  bool have = false;
  for (const pt_light& l : s->lights) have = have || l.type == PT_LIGHT_ENVIRONMENT;
  if (!have) {
    pt_light l{};
    l.type = PT_LIGHT_ENVIRONMENT;
    s->lights.push_back(l);
  }
  return PT_OK;
}

void pt_host_scene_free(pt_host_scene* s) { delete s; }

}  // extern "C"
