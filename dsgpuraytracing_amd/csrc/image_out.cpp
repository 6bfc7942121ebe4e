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
#include <algorithm>
#include <cmath>
#include <cstdint>

#include "pt_error.h"
#include "ptgpu.h"

static inline uint32_t code8(float c) {
  const float one = 1.0f;
  const float m = std::min(std::max(0.0f, one), c);  // clamp(0.f, 1.f, c)
  return (uint32_t)(m * 255);
}

extern "C" int pt_to_color(const float* hdr, int32_t width, int32_t height, int32_t x0, int32_t y0, int32_t x1,
                           int32_t y1, uint32_t* frame) {
  if (!hdr || !frame || width < 0 || height < 0) return pt_fail(PT_E_INVALID, "pt_to_color: bad args");
  x0 = std::max(0, x0);
  y0 = std::max(0, y0);
  x1 = std::min(width, x1);
  y1 = std::min(height, y1);
  const float gamma = 2.2f, level = 1.0f;
  const float one_over_gamma = 1.0f / gamma;
  const float exposure = (float)std::sqrt(std::pow(2, level));
  for (int32_t y = y0; y < y1; ++y)
    for (int32_t x = x0; x < x1; ++x) {
      const float* s = hdr + 3 * ((size_t)x + (size_t)y * (size_t)width);
      const float r = std::pow(s[0] * exposure, one_over_gamma);
      const float g = std::pow(s[1] * exposure, one_over_gamma);
      const float b = std::pow(s[2] * exposure, one_over_gamma);
      frame[(size_t)x + (size_t)y * (size_t)width] = (255u << 24) + (code8(b) << 16) + (code8(g) << 8) + code8(r);
    }
  return PT_OK;
}
