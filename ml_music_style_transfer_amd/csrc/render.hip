// Rendering the model's log-power spectrogram as a complex spectrum with a held phase, for the
// multi-scale spectral loss used as a TRAINING loss (README.md:23, the engel_loss stub at
// model/train.py:119-123):
//
//   X[b][t][f] = M(S[b][f][t]) * U[b][t][f],  M(S) = sqrt(expm1(clip(S, 0, 20)))  (inference.py:109)
//   U = P / |P|  (1 where |P| = 0): the unit phase of a held complex spectrum P (the target's STFT,
//   or the STFT of a Griffin-Lim reconstruction), frame-major like mst_stft_complex_f32's output
//
// and its adjoint dS[b][f][t] = Re(conj(U) dX) * dM/dS with dM/dS = e^S / (2 M) inside (0, 20),
// 0 outside (the clip). The spectrogram is frequency-major (B, F, T), the spectra frame-major
// (B, T, F, 2), so each kernel is a transpose: a 32 (t) x 64 (f) tile goes through LDS, S is read
// along t and the spectra along f, every global access coalesced. HBM-bound elementwise work.
#include "common.h"

namespace {

constexpr int TT = 32, TF = 64;  // tile: 32 frames x 64 bins, 256 threads

__device__ __forceinline__ float2 unit_phase(float2 p) {
  const float r = sqrtf(p.x * p.x + p.y * p.y);
  return r > 0.f ? make_float2(p.x / r, p.y / r) : make_float2(1.f, 0.f);
}

__device__ __forceinline__ float mag_of(float s) {
  return sqrtf(expm1f(fminf(fmaxf(s, 0.f), 20.f)));
}

// grid (ceil(T / TT), ceil(F / TF), B)
__global__ __launch_bounds__(256) void render_fwd_kernel(const float* __restrict__ S,
                                                         const float2* __restrict__ P, int F, int T,
                                                         float2* __restrict__ X) {
  __shared__ float tile[TF][TT + 1];
  const int b = blockIdx.z, t0 = blockIdx.x * TT, f0 = blockIdx.y * TF;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 lanes along t, 8 rows
  const float* Sb = S + (long long)b * F * T;
#pragma unroll
  for (int i = 0; i < TF / 8; ++i) {
    const int f = f0 + ty + 8 * i, t = t0 + tx;
    tile[ty + 8 * i][tx] = (f < F && t < T) ? mag_of(Sb[(long long)f * T + t]) : 0.f;
  }
  __syncthreads();
  const int fx = threadIdx.x & 63, ty2 = threadIdx.x >> 6;  // 64 lanes along f, 4 rows
  const long long base = (long long)b * T * F;
#pragma unroll
  for (int i = 0; i < TT / 4; ++i) {
    const int t = t0 + ty2 + 4 * i, f = f0 + fx;
    if (t < T && f < F) {
      const long long k = base + (long long)t * F + f;
      const float2 u = unit_phase(P[k]);
      const float m = tile[fx][ty2 + 4 * i];
      X[k] = make_float2(m * u.x, m * u.y);
    }
  }
}

__global__ __launch_bounds__(256) void render_bwd_kernel(const float* __restrict__ S,
                                                         const float2* __restrict__ P,
                                                         const float2* __restrict__ dX, int F, int T,
                                                         float* __restrict__ dS) {
  __shared__ float tile[TF][TT + 1];
  const int b = blockIdx.z, t0 = blockIdx.x * TT, f0 = blockIdx.y * TF;
  const int fx = threadIdx.x & 63, ty2 = threadIdx.x >> 6;
  const long long base = (long long)b * T * F;
#pragma unroll
  for (int i = 0; i < TT / 4; ++i) {
    const int t = t0 + ty2 + 4 * i, f = f0 + fx;
    float v = 0.f;
    if (t < T && f < F) {
      const long long k = base + (long long)t * F + f;
      const float2 u = unit_phase(P[k]);
      const float2 g = dX[k];
      v = u.x * g.x + u.y * g.y;  // Re(conj(U) dX)
    }
    tile[fx][ty2 + 4 * i] = v;
  }
  __syncthreads();
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const float* Sb = S + (long long)b * F * T;
  float* dSb = dS + (long long)b * F * T;
#pragma unroll
  for (int i = 0; i < TF / 8; ++i) {
    const int f = f0 + ty + 8 * i, t = t0 + tx;
    if (f < F && t < T) {
      const long long k = (long long)f * T + t;
      const float s = Sb[k];
      float d = 0.f;
      if (s > 0.f && s < 20.f) {
        const float m = sqrtf(expm1f(s));
        d = expf(s) / (2.f * fmaxf(m, 1e-30f));
      }
      dSb[k] = tile[ty + 8 * i][tx] * d;
    }
  }
}

}  // namespace

extern "C" {

int mst_render_logpow_f32(const float* S, const float* P, int32_t B, int32_t F, int32_t T, float* X,
                          void* stream) {
  MST_REQUIRE(S && P && X && B > 0 && F > 0 && T > 0 && B <= 65535);
  MST_REQUIRE((((uintptr_t)P | (uintptr_t)X) & 7) == 0);
  dim3 grid(ceil_div(T, TT), ceil_div(F, TF), B);
  hipLaunchKernelGGL(render_fwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, S,
                     reinterpret_cast<const float2*>(P), F, T, reinterpret_cast<float2*>(X));
  MST_CHECK_LAUNCH();
  return MST_OK;
}

int mst_render_logpow_bwd_f32(const float* S, const float* P, const float* dX, int32_t B, int32_t F,
                              int32_t T, float* dS, void* stream) {
  MST_REQUIRE(S && P && dX && dS && B > 0 && F > 0 && T > 0 && B <= 65535);
  MST_REQUIRE((((uintptr_t)P | (uintptr_t)dX) & 7) == 0);
  dim3 grid(ceil_div(T, TT), ceil_div(F, TF), B);
  hipLaunchKernelGGL(render_bwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, S,
                     reinterpret_cast<const float2*>(P), reinterpret_cast<const float2*>(dX), F, T,
                     dS);
  MST_CHECK_LAUNCH();
  return MST_OK;
}

}  // extern "C"
