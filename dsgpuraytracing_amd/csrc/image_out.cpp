// image_out.cpp — the output row of the path, host side.
//
// HDRImageBuffer::toColor (src/image.h:174-189) + ImageBuffer::update_pixel
// (image.h:49-58), with the reference's arithmetic: exposure =
// sqrt(pow(2, 1.0f)) in double rounded to float, c = std::pow(float, float)
// (glibc powf), code = (uint32_t)(clamp(0.f, 1.f, c) * 255) where CMU462's
// clamp(x, lo, hi) = min(max(x, lo), hi) is called as clamp(0, 1, c), i.e.
// min(1, c): NaN maps to 255 and nothing clamps at 0 (radiance is >= 0).
// Pinned bit for bit against the reference's own toColor by
// tests/test_output.py.
//
// Speed: a channel's 8-bit code is a step function of its value s with 255
// steps, so it is read from a table instead of one powf per channel: code(s)
// for the 2^15 consecutive non-negative floats of one bucket (bits >> 15) is
// the bucket's first code, plus one past the bucket's threshold, if one lies
// inside it.  The thresholds are found with the reference arithmetic itself
// (the smallest float whose code reaches k); negative values, NaN and buckets
// holding two thresholds take the direct powf path.  Exactness rests on
// code(s) being non-decreasing in s; pt_to_color_check compares the table with
// the direct evaluation on every float of a range (tests/test_output.py runs
// it over every float below the 255 threshold).  ~10x faster: the
// asynchronous tile seam (pt_tile_submit) runs it for every completed tile.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "pt_error.h"
#include "ptgpu.h"

namespace {

static inline uint32_t code8(float c) {
  const float one = 1.0f;
  const float m = std::min(std::max(0.0f, one), c);  // clamp(0.f, 1.f, c)
  return (uint32_t)(m * 255);
}

struct ToColor {
  float exposure, one_over_gamma;
  std::vector<uint8_t> code0;    // code at each bucket's first float (buckets = bits >> 15, up to +inf)
  std::vector<uint32_t> inner;   // bits of the threshold inside the bucket (kNone: none)
  std::vector<uint8_t> direct_b; // 1: the bucket holds two thresholds -- powf there
  static constexpr uint32_t kInf = 0x7f800000u, kNone = 0xffffffffu;

  uint32_t direct(float s) const { return code8(std::pow(s * exposure, one_over_gamma)); }
  static float from_bits(uint32_t b) {
    float f;
    std::memcpy(&f, &b, 4);
    return f;
  }
  // smallest bits b in [lo, hi] with direct(b) >= k (hi satisfies it)
  uint32_t first_reaching(uint32_t k, uint32_t lo, uint32_t hi) const {
    while (lo < hi) {
      const uint32_t mid = lo + (hi - lo) / 2;
      if (direct(from_bits(mid)) >= k) hi = mid;
      else lo = mid + 1;
    }
    return lo;
  }
  ToColor() {
    const float gamma = 2.2f, level = 1.0f;
    one_over_gamma = 1.0f / gamma;
    exposure = (float)std::sqrt(std::pow(2, level));
    uint32_t thr[256];
    thr[0] = 0;
    for (uint32_t k = 1; k < 256; ++k) thr[k] = first_reaching(k, thr[k - 1], kInf);
    const uint32_t nb = (kInf >> 15) + 1;
    code0.assign(nb, 0);
    inner.assign(nb, kNone);
    direct_b.assign(nb, 0);
    for (uint32_t b = 0; b < nb; ++b) code0[b] = (uint8_t)direct(from_bits(b << 15));
    for (uint32_t k = 1; k < 256; ++k) {
      const uint32_t b = thr[k] >> 15;
      if ((thr[k] & 0x7fffu) == 0) continue;  // at a bucket start: code0 has it
      if (inner[b] != kNone) direct_b[b] = 1;  // two thresholds in one bucket
      inner[b] = thr[k];
    }
  }
  uint32_t code(float s) const {
    uint32_t b;
    std::memcpy(&b, &s, 4);
    if (b > kInf) return direct(s);  // negatives, NaN
    const uint32_t i = b >> 15;
    if (direct_b[i]) return direct(s);
    return code0[i] + (b >= inner[i] ? 1u : 0u);
  }
};

const ToColor& table() {
  static const ToColor t;  // thread-safe initialisation
  return t;
}

}  // namespace

extern "C" int pt_to_color(const float* hdr, int32_t width, int32_t height, int32_t x0, int32_t y0, int32_t x1,
                           int32_t y1, uint32_t* frame) {
  if (!hdr || !frame || width < 0 || height < 0) return pt_fail(PT_E_INVALID, "pt_to_color: bad args");
  x0 = std::max(0, x0);
  y0 = std::max(0, y0);
  x1 = std::min(width, x1);
  y1 = std::min(height, y1);
  const ToColor& T = table();
  for (int32_t y = y0; y < y1; ++y)
    for (int32_t x = x0; x < x1; ++x) {
      const float* s = hdr + 3 * ((size_t)x + (size_t)y * (size_t)width);
      frame[(size_t)x + (size_t)y * (size_t)width] =
          (255u << 24) + (T.code(s[2]) << 16) + (T.code(s[1]) << 8) + T.code(s[0]);
    }
  return PT_OK;
}

extern "C" int64_t pt_to_color_check(uint32_t lo_bits, uint32_t hi_bits) {
  const ToColor& T = table();
  int64_t bad = 0;
  for (uint64_t b = lo_bits; b < hi_bits; ++b) {
    const float s = ToColor::from_bits((uint32_t)b);
    bad += T.code(s) != T.direct(s);
  }
  return bad;
}
