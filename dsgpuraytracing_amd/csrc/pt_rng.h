// pt_rng.h — counter-based random stream of the HIP path.
//
// The reference draws every random number from glibc std::rand()
// (src/sampler.cpp:14,24-25,35-36,45-46; src/pathtracer.cpp:539; src/bsdf.cpp:147),
// a sequential generator that cannot be replayed in parallel.  The HIP path keys
// an independent stream per (seed, pixel, sample) and consumes it in exactly
// the reference's draw order (camera jitter y then x, per light sample y then x,
// BSDF r1 r2, glass coin, Russian roulette), so a pixel's value is independent
// of scheduling, tile assignment and GPU count.  oracle/restate.cpp (rng_mode=1)
// restates the same function; tests pin the two against each other.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define PT_HD __host__ __device__ __forceinline__
#else
#define PT_HD inline
#endif

namespace ptrng {

PT_HD uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// Per-sample stream base.
PT_HD uint32_t stream_base(uint32_t seed, uint32_t pixel, uint32_t sample) {
  uint32_t h = lowbias32(seed * 0x9E3779B9U ^ pixel);
  return lowbias32(h ^ (sample * 0x85EBCA6BU));
}

// Counter word of draw k: k * kDrawStep + kDrawInit (mod 2^32).  The kernel
// keeps the word itself and adds kDrawStep per draw (no integer multiply,
// a quarter-rate VALU op on CDNA), bit-identical to draw(base, k).
constexpr uint32_t kDrawStep = 0xC2B2AE35U, kDrawInit = 0x27D4EB2FU;

// The draw with counter word kc as a 24-bit uniform in [0, 1), exact in float.
PT_HD float draw_at(uint32_t base, uint32_t kc) {
  uint32_t h = lowbias32(base ^ kc);
  return (float)(h >> 8) * (1.0f / 16777216.0f);
}

// Draw k of a stream.
PT_HD float draw(uint32_t base, uint32_t k) { return draw_at(base, k * kDrawStep + kDrawInit); }

}  // namespace ptrng
