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

// Draw k of a stream as a 24-bit uniform in [0, 1), exact in float.
PT_HD float draw(uint32_t base, uint32_t k) {
  uint32_t h = lowbias32(base ^ (k * 0xC2B2AE35U + 0x27D4EB2FU));
  return (float)(h >> 8) * (1.0f / 16777216.0f);
}

}  // namespace ptrng
