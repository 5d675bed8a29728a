// Shared device helpers for libmst_hip (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mst.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define MST_CHECK_LAUNCH()                                  \
  do {                                                      \
    hipError_t e_ = hipGetLastError();                      \
    if (e_ != hipSuccess) return -(int)e_;                  \
  } while (0)

#define MST_REQUIRE(cond)            \
  do {                               \
    if (!(cond)) return MST_EINVAL;  \
  } while (0)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// splitmix64 finaliser -> 32 bits; dropout keep test is hash >= p * 2^32.
__device__ __forceinline__ uint32_t mst_hash32(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + idx * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}

__device__ __forceinline__ float lrelu(float x, float s) { return x > 0.f ? x : x * s; }

// cos / sin of 2 pi m / n in double, evaluated at compile time (quadrant-reduced Taylor series)
static constexpr double kPiD = 3.14159265358979323846264338327950288;
static constexpr void cx_sincos_turn(long long m, long long n, double& c, double& s) {
  m %= n;
  if (m < 0) m += n;
  const long long q = (4 * m) / n;                 // quadrant
  const double x = (double)(4 * m - q * n) / (double)n * (kPiD / 2);  // [0, pi/2)
  double x2 = x * x, ts = x, ss = x, tc = 1.0, sc = 1.0;
  for (int k = 1; k < 16; ++k) {
    ts *= -x2 / ((2.0 * k) * (2.0 * k + 1.0));
    ss += ts;
    tc *= -x2 / ((2.0 * k - 1.0) * (2.0 * k));
    sc += tc;
  }
  const double cq[4] = {sc, -ss, -sc, ss}, sq[4] = {ss, sc, -ss, -sc};
  c = cq[q];
  s = sq[q];
}

static inline int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }
