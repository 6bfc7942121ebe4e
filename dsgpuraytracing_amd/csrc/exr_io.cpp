// exr_io.cpp — native OpenEXR reader for environment maps (host side).
//
// Replaces the reference's `-e` path: load_exr (src/main.cpp:30-67) over the
// vendored tinyexr (CMU462/include/CMU462/tinyexr.h, ParseMultiChannelEXRHeader
// FromFile + LoadMultiChannelEXRFromFile).  Supported: single-part scanline
// files, compression NONE (0), ZIPS (2) and ZIP (3) (zlib + the OpenEXR
// predictor/interleave transform), channel types HALF and FLOAT.  The
// reference's channel mapping is kept on purpose: it reads the file's
// (name-sorted) channels by index as R = channel 2, G = channel 1, B =
// channel 0, which is right for B,G,R files and shifts colours for A,B,G,R
// ones (main.cpp:53-55).  PIZ and other codecs are rejected with PT_E_IO.
#include <zlib.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ptgpu_scene.h"
#include "pt_error.h"

namespace {

float half_to_float(uint16_t h) {
  const uint32_t s = (uint32_t)(h >> 15) << 31;
  const uint32_t e = (h >> 10) & 0x1f;
  const uint32_t m = h & 0x3ff;
  uint32_t bits;
  if (e == 0) {
    if (m == 0) {
      bits = s;
    } else {  // subnormal half -> normal float
      int ee = -1;
      uint32_t mm = m;
      do {
        ++ee;
        mm <<= 1;
      } while ((mm & 0x400) == 0);
      bits = s | ((uint32_t)(127 - 15 - ee) << 23) | ((mm & 0x3ff) << 13);
    }
  } else if (e == 31) {
    bits = s | 0x7f800000u | (m << 13);
  } else {
    bits = s | ((e + 127 - 15) << 23) | (m << 13);
  }
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

struct Channel {
  std::string name;
  int type;  // 0 UINT, 1 HALF, 2 FLOAT
};

struct Reader {
  const std::vector<uint8_t>& b;
  size_t p = 0;
  bool bad = false;
  explicit Reader(const std::vector<uint8_t>& buf) : b(buf) {}
  bool have(size_t n) {
    if (p + n > b.size()) bad = true;
    return !bad;
  }
  std::string cstr() {
    std::string s;
    while (have(1) && b[p] != 0) s.push_back((char)b[p++]);
    if (have(1)) ++p;
    return s;
  }
  template <class T>
  T get() {
    T v{};
    if (have(sizeof(T))) {
      std::memcpy(&v, &b[p], sizeof(T));
      p += sizeof(T);
    }
    return v;
  }
};

// OpenEXR ZIP/ZIPS block: zlib, then undo the byte predictor and the
// even/odd interleave.
bool unzip_block(const uint8_t* src, size_t n, std::vector<uint8_t>& out, size_t expect) {
  std::vector<uint8_t> tmp(expect);
  uLongf len = (uLongf)expect;
  if (uncompress(tmp.data(), &len, src, (uLong)n) != Z_OK || len != expect) return false;
  for (size_t i = 1; i < expect; ++i) tmp[i] = (uint8_t)(tmp[i - 1] + tmp[i] - 128);
  out.resize(expect);
  const size_t half = (expect + 1) / 2;
  for (size_t i = 0; i < expect; ++i) out[i] = (i & 1) ? tmp[half + i / 2] : tmp[i / 2];
  return true;
}

int load(const char* path, int32_t* W, int32_t* H, float** rgb_out) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return pt_fail(PT_E_IO, std::string("pt_host_load_exr: cannot open ") + path);
  std::vector<uint8_t> buf;
  {
    uint8_t tmp[1 << 16];
    size_t n;
    while ((n = std::fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + n);
    std::fclose(f);
  }
  Reader r(buf);
  if (r.get<int32_t>() != 20000630) return pt_fail(PT_E_IO, "pt_host_load_exr: not an OpenEXR file");
  const int32_t version = r.get<int32_t>();
  if ((version & 0xff) != 2 || (version & 0x1e00) != 0)  // tiled / deep / multi-part
    return pt_fail(PT_E_IO, "pt_host_load_exr: only single-part scanline files are supported");
  std::vector<Channel> ch;
  int comp = -1;
  int32_t dw[4] = {0, 0, -1, -1};
  for (;;) {
    std::string name = r.cstr();
    if (r.bad) return pt_fail(PT_E_IO, "pt_host_load_exr: truncated header");
    if (name.empty()) break;
    std::string type = r.cstr();
    int32_t size = r.get<int32_t>();
    if (r.bad || size < 0 || !r.have((size_t)size)) return pt_fail(PT_E_IO, "pt_host_load_exr: truncated header");
    size_t end = r.p + (size_t)size;
    if (name == "channels") {
      while (r.p < end) {
        std::string cn = r.cstr();
        if (cn.empty()) break;
        Channel c;
        c.name = cn;
        c.type = r.get<int32_t>();
        r.p += 4;                  // pLinear + reserved
        int32_t xs = r.get<int32_t>(), ys = r.get<int32_t>();
        if (xs != 1 || ys != 1) return pt_fail(PT_E_IO, "pt_host_load_exr: subsampled channels are not supported");
        ch.push_back(c);
      }
    } else if (name == "compression") {
      comp = buf[r.p];
    } else if (name == "dataWindow") {
      std::memcpy(dw, &buf[r.p], 16);
    }
    r.p = end;
  }
  if (ch.size() < 3) return pt_fail(PT_E_IO, "pt_host_load_exr: fewer than 3 channels (load_exr reads channels 0-2)");
  for (const Channel& c : ch)
    if (c.type != 1 && c.type != 2) return pt_fail(PT_E_IO, "pt_host_load_exr: only HALF and FLOAT channels are supported");
  if (comp != 0 && comp != 2 && comp != 3)
    return pt_fail(PT_E_IO, "pt_host_load_exr: compression " + std::to_string(comp) + " is not supported (NONE, ZIPS, ZIP)");
  const int64_t w = (int64_t)dw[2] - dw[0] + 1, h = (int64_t)dw[3] - dw[1] + 1;
  if (w <= 0 || h <= 0 || w * h > ((int64_t)1 << 31)) return pt_fail(PT_E_IO, "pt_host_load_exr: bad data window");
  const int lines = comp == 3 ? 16 : 1;
  const int64_t nblocks = (h + lines - 1) / lines;
  std::vector<uint64_t> offs((size_t)nblocks);
  for (auto& o : offs) o = r.get<uint64_t>();
  if (r.bad) return pt_fail(PT_E_IO, "pt_host_load_exr: truncated offset table");
  size_t line_bytes = 0;
  for (const Channel& c : ch) line_bytes += (size_t)w * (c.type == 1 ? 2 : 4);
  std::vector<std::vector<float>> img(ch.size(), std::vector<float>((size_t)(w * h)));
  std::vector<uint8_t> raw;
  for (int64_t bi = 0; bi < nblocks; ++bi) {
    Reader br(buf);
    br.p = (size_t)offs[(size_t)bi];
    const int32_t y = br.get<int32_t>();
    const int32_t n = br.get<int32_t>();
    if (br.bad || n < 0 || !br.have((size_t)n)) return pt_fail(PT_E_IO, "pt_host_load_exr: truncated block");
    const int64_t y0 = (int64_t)y - dw[1];
    if (y0 < 0 || y0 >= h) return pt_fail(PT_E_IO, "pt_host_load_exr: block outside the data window");
    const int64_t ny = std::min<int64_t>(lines, h - y0);
    const size_t expect = line_bytes * (size_t)ny;
    const uint8_t* data = &buf[br.p];
    if ((size_t)n == expect) {  // stored uncompressed (also allowed inside ZIP files)
      raw.assign(data, data + expect);
    } else if (comp == 0 || !unzip_block(data, (size_t)n, raw, expect)) {
      return pt_fail(PT_E_IO, "pt_host_load_exr: corrupt block");
    }
    size_t q = 0;
    for (int64_t yy = 0; yy < ny; ++yy)
      for (size_t c = 0; c < ch.size(); ++c) {
        float* dst = &img[c][(size_t)((y0 + yy) * w)];
        if (ch[c].type == 1) {
          for (int64_t x = 0; x < w; ++x, q += 2) {
            uint16_t v;
            std::memcpy(&v, &raw[q], 2);
            dst[x] = half_to_float(v);
          }
        } else {
          std::memcpy(dst, &raw[q], (size_t)w * 4);
          q += (size_t)w * 4;
        }
      }
  }
  float* out = (float*)std::malloc((size_t)(w * h) * 3 * sizeof(float));
  if (!out) return pt_fail(PT_E_ALLOC, "pt_host_load_exr: out of memory");
  for (int64_t i = 0; i < w * h; ++i) {  // main.cpp:53-61
    out[3 * i] = img[2][(size_t)i];
    out[3 * i + 1] = img[1][(size_t)i];
    out[3 * i + 2] = img[0][(size_t)i];
  }
  *W = (int32_t)w;
  *H = (int32_t)h;
  *rgb_out = out;
  return PT_OK;
}

}  // namespace

extern "C" {

int pt_host_load_exr(const char* path, int32_t* width, int32_t* height, float** rgb) {
  if (!path || !width || !height || !rgb) return pt_fail(PT_E_INVALID, "pt_host_load_exr: NULL argument");
  *rgb = nullptr;
  return load(path, width, height, rgb);
}

void pt_host_free(void* p) { std::free(p); }

}  // extern "C"
