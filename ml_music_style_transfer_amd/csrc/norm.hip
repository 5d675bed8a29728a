// Bandwidth-bound kernels of the training step (one wave per NCL row where a row reduction
// is needed):
//   InstanceNorm1d(eps=1e-5, no affine) + LeakyReLU(0.01) [+ MaxPool1d(2,2)] fwd/bwd
//       model/model.py:40-53 (DownConv), 65-69 + 81-89 (UpConv)
//   bias gradients (sum over batch and time)
//   lrelu(lastconv) + L1 loss fwd/bwd   model/model.py:299, model/train.py:132-135,140
//   Adam over the flat parameter buffer  model/train.py:188,143
//   piano-roll binarise + onset/offset   preprocessing/preprocess.py:148-155
#include <cstdlib>

#include "common.h"

namespace {

// ---------------------------------------------------------------------------
// InstanceNorm + LeakyReLU (+ MaxPool) forward. G lanes per row (a wave, or for short rows
// (T <= 2 G < 128) a G-lane segment of one, so several rows share a wave); lane l holds the
// element pairs (2l + 2Gp, 2l + 2Gp + 1), p < NP, so the pool pairs are lane-local.
// Two-pass (exact) mean/variance in registers; biased variance like torch.
// ---------------------------------------------------------------------------
// sum over the G-lane segment of a wave (G = 64: wave_sum's order)
template <int G>
__device__ __forceinline__ float seg_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t in_rsrc(const float* base, long long n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0,
                                           base ? (int)(4 * n) : 0, 0x00020000);
}
__device__ __forceinline__ float in_ld(__amdgpu_buffer_rsrc_t rs, long long i) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(4 * i), 0, 0));
}
// elements i, i + 1 (i even, 8-byte aligned) in one load
__device__ __forceinline__ float2 in_ld2(__amdgpu_buffer_rsrc_t rs, long long i) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(4 * i), 0, 0);
  return make_float2(__uint_as_float(v[0]), __uint_as_float(v[1]));
}

// EVEN (T even, every base 8-byte aligned): a lane's element pair is one 8-byte load and one
// 8-byte store, in or out of the row together. All loads are issued before any is used, from
// clamped in-row addresses (a load-or-default branch per element makes hipcc wait at each join).
template <int NP, int G, bool EVEN>
__global__ __launch_bounds__(256) void in_fwd_kernel(const float* __restrict__ y, long long rows,
                                                     int T, float eps, float slope,
                                                     float* __restrict__ a, float* __restrict__ pooled,
                                                     float* __restrict__ mean,
                                                     float* __restrict__ rstd) {
  const long long row = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / G;
  const int lane = threadIdx.x & (G - 1);
  if (row >= rows) return;
  const auto ry = in_rsrc(y, rows * T);
  float e0[NP], e1[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int i0 = 2 * lane + 2 * G * q;
    if constexpr (EVEN) {
      const float2 v = in_ld2(ry, row * T + (i0 < T ? i0 : 0));
      e0[q] = v.x;
      e1[q] = v.y;
    } else {
      e0[q] = in_ld(ry, row * T + (i0 < T ? i0 : 0));
      e1[q] = in_ld(ry, row * T + (i0 + 1 < T ? i0 + 1 : 0));
    }
  }
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int i0 = 2 * lane + 2 * G * q;
    e0[q] = i0 < T ? e0[q] : 0.f;
    e1[q] = i0 + 1 < T ? e1[q] : 0.f;
    s += e0[q] + e1[q];
  }
  s = seg_sum<G>(s);
  const float mu = s / (float)T;
  float v = 0.f;
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    int i0 = 2 * lane + 2 * G * q;
    float d0 = e0[q] - mu, d1 = e1[q] - mu;
    if (i0 < T) v += d0 * d0;
    if (i0 + 1 < T) v += d1 * d1;
  }
  v = seg_sum<G>(v);
  const float r = 1.f / sqrtf(v / (float)T + eps);
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = r;
  }
  float* ar = a + row * T;
  const int Tp = T >> 1;
  float* pr = pooled ? pooled + row * Tp : nullptr;
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    int i0 = 2 * lane + 2 * G * q;
    float a0 = lrelu((e0[q] - mu) * r, slope);
    float a1 = lrelu((e1[q] - mu) * r, slope);
    if constexpr (EVEN) {
      if (i0 < T) *reinterpret_cast<float2*>(ar + i0) = make_float2(a0, a1);
    } else {
      if (i0 < T) ar[i0] = a0;
      if (i0 + 1 < T) ar[i0 + 1] = a1;
    }
    if (pr && (i0 >> 1) < Tp) pr[i0 >> 1] = (a1 > a0) ? a1 : a0;  // first index wins ties
  }
}

// Long rows (T > 128*16): three streaming passes over global memory.
__global__ __launch_bounds__(256) void in_fwd_long_kernel(const float* __restrict__ y,
                                                          long long rows, int T, float eps,
                                                          float slope, float* __restrict__ a,
                                                          float* __restrict__ pooled,
                                                          float* __restrict__ mean,
                                                          float* __restrict__ rstd) {
  const long long row = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* yr = y + row * T;
  float s = 0.f;
  for (int i = lane; i < T; i += 64) s += yr[i];
  const float mu = wave_sum(s) / (float)T;
  float v = 0.f;
  for (int i = lane; i < T; i += 64) {
    float d = yr[i] - mu;
    v += d * d;
  }
  const float r = 1.f / sqrtf(wave_sum(v) / (float)T + eps);
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = r;
  }
  float* ar = a + row * T;
  const int Tp = T >> 1;
  for (int i0 = 2 * lane; i0 < T; i0 += 128) {
    float a0 = lrelu((yr[i0] - mu) * r, slope);
    ar[i0] = a0;
    if (i0 + 1 < T) {
      float a1 = lrelu((yr[i0 + 1] - mu) * r, slope);
      ar[i0 + 1] = a1;
      if (pooled && (i0 >> 1) < Tp) pooled[row * Tp + (i0 >> 1)] = (a1 > a0) ? a1 : a0;
    }
  }
}

// Backward: da = d_a + unpool(d_pool0 + d_pool1) (to the pair's argmax), dz = lrelu'(z) da,
// dy = rstd * (dz - mean(dz) - z * mean(dz * z)).
template <int NP, int G, bool EVEN>
__global__ __launch_bounds__(256) void in_bwd_kernel(const float* __restrict__ y,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ rstd,
                                                     long long rows, int T, float slope,
                                                     const float* __restrict__ d_a,
                                                     const float* __restrict__ dp0,
                                                     const float* __restrict__ dp1,
                                                     float* __restrict__ dy,
                                                     float* __restrict__ rowsum) {
  const long long row = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / G;
  const int lane = threadIdx.x & (G - 1);
  if (row >= rows) return;
  const float mu = mean[row], r = rstd[row];
  const int Tp = T >> 1;
  float z0[NP], z1[NP], g0[NP], g1[NP];
  float s1 = 0.f, s2 = 0.f;
  // every load of the row is issued before any is used, from clamped in-row addresses (a
  // per-element "load or default" branch made the compiler wait vmcnt(0) at each join: five
  // serialised round trips per row, 2.2 TB/s against the forward kernel's 6.4)
  // whole-tensor buffer descriptors (wave-uniform: a per-row descriptor is not, and hipcc wraps
  // each load in a waterfall loop); an absent input (null) reads 0 through the range check;
  // element indices are clamped into the row and the values past it masked below
  const auto ry = in_rsrc(y, rows * T), ra = in_rsrc(d_a, rows * T);
  const auto rp0 = in_rsrc(dp0, rows * Tp), rp1 = in_rsrc(dp1, rows * Tp);
  const bool has_p = (dp0 || dp1) && Tp > 0;  // kernel-uniform
  float y0v[NP], y1v[NP], a0v[NP], a1v[NP], gpv[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int i0 = 2 * lane + 2 * G * q;
    const long long e0 = row * T + (i0 < T ? i0 : 0), e1 = row * T + (i0 + 1 < T ? i0 + 1 : 0);
    const long long ep = row * Tp + ((i0 >> 1) < Tp ? (i0 >> 1) : 0);
    if constexpr (EVEN) {
      const float2 yv = in_ld2(ry, e0), av = in_ld2(ra, e0);
      y0v[q] = yv.x;
      y1v[q] = yv.y;
      a0v[q] = av.x;
      a1v[q] = av.y;
    } else {
      y0v[q] = in_ld(ry, e0);
      y1v[q] = in_ld(ry, e1);
      a0v[q] = in_ld(ra, e0);
      a1v[q] = in_ld(ra, e1);
    }
    gpv[q] = in_ld(rp0, ep) + in_ld(rp1, ep);
  }
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int i0 = 2 * lane + 2 * G * q;
    const bool ok0 = i0 < T, ok1 = i0 + 1 < T;
    z0[q] = ((ok0 ? y0v[q] : mu) - mu) * r;
    z1[q] = ((ok1 ? y1v[q] : mu) - mu) * r;
    float da0 = ok0 ? a0v[q] : 0.f, da1 = ok1 ? a1v[q] : 0.f;
    if (has_p && (i0 >> 1) < Tp) {
      const float a0 = lrelu(z0[q], slope), a1 = lrelu(z1[q], slope);
      if (a1 > a0) da1 += gpv[q];
      else da0 += gpv[q];
    }
    g0[q] = ok0 ? (z0[q] > 0.f ? da0 : da0 * slope) : 0.f;
    g1[q] = ok1 ? (z1[q] > 0.f ? da1 : da1 * slope) : 0.f;
    s1 += g0[q] + g1[q];
    s2 += g0[q] * z0[q] + g1[q] * z1[q];
  }
  s1 = seg_sum<G>(s1) / (float)T;
  s2 = seg_sum<G>(s2) / (float)T;
  float* dr = dy + row * T;
  float rs = 0.f;
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    int i0 = 2 * lane + 2 * G * q;
    const float v0 = r * (g0[q] - s1 - z0[q] * s2), v1 = r * (g1[q] - s1 - z1[q] * s2);
    if constexpr (EVEN) {
      if (i0 < T) {
        *reinterpret_cast<float2*>(dr + i0) = make_float2(v0, v1);
        rs += v0;
        rs += v1;
      }
    } else {
      if (i0 < T) {
        dr[i0] = v0;
        rs += v0;
      }
      if (i0 + 1 < T) {
        dr[i0 + 1] = v1;
        rs += v1;
      }
    }
  }
  if (rowsum) {
    rs = seg_sum<G>(rs);
    if (lane == 0) rowsum[row] = rs;
  }
}

__device__ __forceinline__ float in_bwd_g(const float* yr, int i, int T, int Tp, float mu, float r,
                                          float slope, const float* da_r, const float* dp0r,
                                          const float* dp1r, float* zout) {
  float z = (yr[i] - mu) * r;
  *zout = z;
  float da = da_r ? da_r[i] : 0.f;
  int pi = i >> 1;
  if ((dp0r || dp1r) && pi < Tp) {
    int j = i ^ 1;
    float zo = (yr[j] - mu) * r;
    float a = lrelu(z, slope), ao = lrelu(zo, slope);
    bool second_wins = (i & 1) ? (a > ao) : (ao > a);
    bool mine = (i & 1) ? second_wins : !second_wins;
    if (mine) da += (dp0r ? dp0r[pi] : 0.f) + (dp1r ? dp1r[pi] : 0.f);
  }
  return z > 0.f ? da : da * slope;
}

__global__ __launch_bounds__(256) void in_bwd_long_kernel(const float* __restrict__ y,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ rstd,
                                                          long long rows, int T, float slope,
                                                          const float* __restrict__ d_a,
                                                          const float* __restrict__ dp0,
                                                          const float* __restrict__ dp1,
                                                          float* __restrict__ dy,
                                                          float* __restrict__ rowsum) {
  const long long row = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* yr = y + row * T;
  const float mu = mean[row], r = rstd[row];
  const int Tp = T >> 1;
  const float* dar = d_a ? d_a + row * T : nullptr;
  const float* p0 = dp0 ? dp0 + row * Tp : nullptr;
  const float* p1 = dp1 ? dp1 + row * Tp : nullptr;
  float s1 = 0.f, s2 = 0.f;
  for (int i = lane; i < T; i += 64) {
    float z;
    float g = in_bwd_g(yr, i, T, Tp, mu, r, slope, dar, p0, p1, &z);
    s1 += g;
    s2 += g * z;
  }
  s1 = wave_sum(s1) / (float)T;
  s2 = wave_sum(s2) / (float)T;
  float rs = 0.f;
  for (int i = lane; i < T; i += 64) {
    float z;
    float g = in_bwd_g(yr, i, T, Tp, mu, r, slope, dar, p0, p1, &z);
    const float v = r * (g - s1 - z * s2);
    dy[row * T + i] = v;
    rs += v;
  }
  if (rowsum) {
    rs = wave_sum(rs);
    if (lane == 0) rowsum[row] = rs;
  }
}

// db[c] = scale * sum_b rowsum[b * C + c] (+ db[c]): the bias gradient from per-row sums.
__global__ __launch_bounds__(256) void bias_rows_kernel(const float* __restrict__ rowsum, int B,
                                                        int C, float scale, float* __restrict__ db,
                                                        int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
#pragma unroll 8
  for (int b = 0; b < B; ++b) s += rowsum[(long long)b * C + c];
  s *= scale;
  db[c] = accumulate ? db[c] + s : s;
}

// db[c] = scale * sum_{b,t} dy[b][c][t] (+ db[c]); one 256-thread workgroup per channel over the
// flattened (b, t) index j = b T + t: thread k sums j = k, k + 256, ... (coalesced within each
// row, every thread busy whatever T is), then a fixed-order wave and workgroup reduction
// (deterministic). Round 3's one-wave-per-channel form had a single wave walk all B rows of a
// channel (34 us per call at 14 calls per step, latency-bound).
__global__ __launch_bounds__(256) void bias_grad_kernel(const float* __restrict__ dy, int B, int C,
                                                        int T, float scale, float* __restrict__ db,
                                                        int accumulate) {
  __shared__ float part[4];
  const int c = blockIdx.x;
  const int n = B * T;
  float s0 = 0.f, s1 = 0.f;
  int j = threadIdx.x;
  for (; j + 256 < n; j += 512) {  // two independent chains
    const int b0 = j / T, b1 = (j + 256) / T;
    s0 += dy[((long long)b0 * C + c) * T + (j - b0 * T)];
    s1 += dy[((long long)b1 * C + c) * T + (j + 256 - b1 * T)];
  }
  if (j < n) {
    const int b0 = j / T;
    s0 += dy[((long long)b0 * C + c) * T + (j - b0 * T)];
  }
  const float s = wave_sum(s0 + s1);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float v = ((part[0] + part[1]) + (part[2] + part[3])) * scale;
    if (accumulate) v += db[c];
    db[c] = v;
  }
}

// ---------------------------------------------------------------------------
// L1 / MSE loss: per-block double partials, then one block finishes (deterministic).
// ---------------------------------------------------------------------------
template <int MODE>  // 1: L1(pred, t), 2: MSE(pred, t)
__global__ __launch_bounds__(256) void loss_partial_kernel(const float* __restrict__ x,
                                                           const float* __restrict__ t,
                                                           long long n, double* __restrict__ part) {
  double s = 0.0;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    float d = x[i] - t[i];
    s += (MODE == 2) ? (double)d * d : (double)fabsf(d);
  }
  __shared__ double red[4];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void loss_final_kernel(const double* __restrict__ part, int nb,
                                                         long long n, float* __restrict__ loss) {
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) s += part[i];
  __shared__ double red[4];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) loss[0] = (float)((red[0] + red[1] + red[2] + red[3]) / (double)n);
}

// Adam (torch.optim.Adam, single-tensor formulation): m.lerp_(g, 1-b1); v = v*b2 + (1-b2) g^2;
// p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps). Vectorised 4-wide over the flat buffer; UNR float4
// groups per thread per grid-stride step (all loads issued before the arithmetic, so UNR x 4
// 16-byte loads are in flight per lane). NT: nontemporal loads/stores (streamed once).
// hyper (nullable, device) = {lr/bc1, sqrt(bc2)} overrides the by-value pair: a captured
// hipGraph replays one launch whose step-dependent factors the graph itself computes.
template <int UNR, bool NT>
__device__ __forceinline__ f32x4 adam_ld(const f32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <int UNR, bool NT>
__device__ __forceinline__ void adam_st(f32x4 v, f32x4* p) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
template <int UNR, bool NT>
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   long long n, float lr_step, float b2, float w1,
                                                   float w2, float eps, float bc2_sqrt,
                                                   const float* __restrict__ hyper) {
  if (hyper) {
    lr_step = hyper[0];
    bc2_sqrt = hyper[1];
  }
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  f32x4* P = reinterpret_cast<f32x4*>(p);
  const f32x4* G = reinterpret_cast<const f32x4*>(g);
  f32x4* M = reinterpret_cast<f32x4*>(m);
  f32x4* V = reinterpret_cast<f32x4*>(v);
  for (long long i0 = (long long)blockIdx.x * blockDim.x + threadIdx.x; i0 < n4; i0 += UNR * stride) {
    f32x4 pv[UNR], gv[UNR], mv[UNR], vv[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const long long i = i0 + u * stride;
      if (UNR == 1 || i < n4) {
        pv[u] = adam_ld<UNR, NT>(P + i);
        gv[u] = adam_ld<UNR, NT>(G + i);
        mv[u] = adam_ld<UNR, NT>(M + i);
        vv[u] = adam_ld<UNR, NT>(V + i);
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const long long i = i0 + u * stride;
      if (UNR > 1 && i >= n4) break;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        mv[u][k] = mv[u][k] + w1 * (gv[u][k] - mv[u][k]);
        vv[u][k] = vv[u][k] * b2 + w2 * (gv[u][k] * gv[u][k]);
        float den = sqrtf(vv[u][k]) / bc2_sqrt + eps;
        pv[u][k] = pv[u][k] - lr_step * (mv[u][k] / den);
      }
      adam_st<UNR, NT>(pv[u], P + i);
      adam_st<UNR, NT>(mv[u], M + i);
      adam_st<UNR, NT>(vv[u], V + i);
    }
  }
  // tail
  long long i = (n4 << 2) + (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && i < n) {
    float gs = g[i], ms = m[i], vs = v[i];
    ms = ms + w1 * (gs - ms);
    vs = vs * b2 + w2 * (gs * gs);
    float den = sqrtf(vs) / bc2_sqrt + eps;
    p[i] = p[i] - lr_step * (ms / den);
    m[i] = ms;
    v[i] = vs;
  }
}

// A/B knob (read once): MST_ADAM_VARIANT = "<unroll><n|p>" (nontemporal / plain), default 2n
// (tools/adam_micro.py over the bench's 726 M parameters: 1n 3.83 ms, 2n 3.52 ms, 4n 3.86 ms,
// 2p 4.05 ms at 16384 workgroups; profiles/r03/adam_micro_m1.jsonl); MST_ADAM_BLOCKS caps the
// default grid (16384)
struct AdamCfg {
  int unr = 2;
  bool nt = true;
  int blocks = 16384;
};
static const AdamCfg& adam_cfg() {
  static const AdamCfg c = [] {
    AdamCfg r;
    if (const char* e = getenv("MST_ADAM_VARIANT")) {
      if (e[0] >= '1' && e[0] <= '4') r.unr = e[0] - '0';
      if (e[0] && e[1] == 'p') r.nt = false;
    }
    if (const char* e = getenv("MST_ADAM_BLOCKS")) r.blocks = atoi(e) > 0 ? atoi(e) : r.blocks;
    return r;
  }();
  return c;
}
static void launch_adam(dim3 grid, hipStream_t st, float* p, const float* g, float* m, float* v,
                        long long n, float lr_step, float b2, float w1, float w2, float eps,
                        float bc2_sqrt, const float* hyper) {
  const AdamCfg& c = adam_cfg();
#define MST_ADAM_L(U, NTF) hipLaunchKernelGGL((adam_kernel<U, NTF>), grid, dim3(256), 0, st, p, g, m, v, n, lr_step, b2, w1, w2, eps, bc2_sqrt, hyper)
  if (c.nt) {
    if (c.unr == 1) MST_ADAM_L(1, true);
    else if (c.unr == 2) MST_ADAM_L(2, true);
    else MST_ADAM_L(4, true);
  } else {
    if (c.unr == 1) MST_ADAM_L(1, false);
    else if (c.unr == 2) MST_ADAM_L(2, false);
    else MST_ADAM_L(4, false);
  }
#undef MST_ADAM_L
}

__global__ void scale_kernel(float* x, long long n, float s) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    x[i] *= s;
}

__global__ void fill_kernel(float* x, long long n, float v) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    x[i] = v;
}

// preprocess.py:148-155: bin = roll != 0; onoff[t] = bin[t] - bin[t-1] (bin[-1] = 0).
__global__ void onoff_kernel(const float* __restrict__ roll, int B, int T, float* __restrict__ bin,
                             float* __restrict__ onoff) {
  long long n = (long long)B * T * 128;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    int t = (int)((i / 128) % T);
    float cur = roll[i] != 0.f ? 1.f : 0.f;
    float prev = (t > 0 && roll[i - 128] != 0.f) ? 1.f : 0.f;
    bin[i] = cur;
    onoff[i] = cur - prev;
  }
}

// dx = gscale[0]/n * sign(pred - t)   (nn.L1Loss backward; sign(0) = 0)
__global__ void l1_bwd_kernel(const float* __restrict__ pred, const float* __restrict__ t,
                              long long n, const float* __restrict__ gscale, float* __restrict__ dx) {
  const float g = (gscale ? gscale[0] : 1.f) / (float)n;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    float d = pred[i] - t[i];
    dx[i] = d > 0.f ? g : (d < 0.f ? -g : 0.f);
  }
}

// dx = dy * (y > 0 ? 1 : slope)   (LeakyReLU backward from its output's sign)
__global__ void lrelu_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                 long long n, float slope, float* __restrict__ dx) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    float g = dy[i];
    dx[i] = y[i] > 0.f ? g : g * slope;
  }
}

// out = h > 0 ? d * s : 0   (ReLU + inverted-dropout backward from the kept output h)
__global__ void relu_gate_bwd_kernel(const float* __restrict__ d, const float* __restrict__ h,
                                     long long n, float s, float* __restrict__ out) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    out[i] = h[i] > 0.f ? d[i] * s : 0.f;
}

// lanes per InstanceNorm row: two elements per lane, a power of two in [4, 64] (short rows share
// a wave instead of leaving most of its lanes idle); MST_IN_SEG=0 keeps one row per wave (A/B)
int in_lanes(int T) {
  static const bool seg = [] {
    const char* e = getenv("MST_IN_SEG");
    return !(e && e[0] == '0');
  }();
  if (!seg) return 64;
  int g = 4;
  while (g < 64 && 2 * g < T) g *= 2;
  return g;
}

int grid_for(long long n, int per = 256, int cap = 8192) {
  long long g = (n + per - 1) / per;
  if (g > cap) g = cap;
  return g < 1 ? 1 : (int)g;
}

}  // namespace

extern "C" {

int mst_instnorm_lrelu_fwd_f32(const float* y, int64_t rows, int32_t T, float eps, float slope,
                               float* a, float* pooled, float* mean, float* rstd, void* stream) {
  MST_REQUIRE(y && a && mean && rstd && rows > 0 && T > 1);
  // in_fwd_kernel addresses through 32-bit buffer byte offsets; larger tensors take the
  // long-row kernel (64-bit addressing)
  const bool buf32 = rows * (long long)T < (1ll << 29);
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  int np = (T + 127) / 128;
  const int g = in_lanes(T);
  dim3 gs((unsigned)((rows * g + 255) / 256));
  const bool even = T % 2 == 0 && (((uintptr_t)y | (uintptr_t)a) & 7) == 0;
#define MST_IN(NP_, G_, GR)                                                                            \
  do {                                                                                                 \
    if (even) hipLaunchKernelGGL((in_fwd_kernel<NP_, G_, true>), GR, block, 0, st, y, rows, T, eps, slope, a, pooled, mean, rstd); \
    else hipLaunchKernelGGL((in_fwd_kernel<NP_, G_, false>), GR, block, 0, st, y, rows, T, eps, slope, a, pooled, mean, rstd); \
  } while (0)
  if (buf32 && np <= 1 && g < 64) {
    if (g == 4) MST_IN(1, 4, gs);
    else if (g == 8) MST_IN(1, 8, gs);
    else if (g == 16) MST_IN(1, 16, gs);
    else MST_IN(1, 32, gs);
  } else if (buf32 && np <= 1) MST_IN(1, 64, grid);
  else if (buf32 && np <= 2) MST_IN(2, 64, grid);
  else if (buf32 && np <= 4) MST_IN(4, 64, grid);
  else if (buf32 && np <= 8) MST_IN(8, 64, grid);
#undef MST_IN
  else hipLaunchKernelGGL(in_fwd_long_kernel, grid, block, 0, st, y, rows, T, eps, slope, a, pooled, mean, rstd);
  MST_CHECK_LAUNCH();
  return MST_OK;
}

int mst_instnorm_lrelu_bwd_f32(const float* y, const float* mean, const float* rstd, int64_t rows,
                               int32_t T, float slope, const float* d_a, const float* d_pool0,
                               const float* d_pool1, float* dy, float* rowsum, void* stream) {
  MST_REQUIRE(y && mean && rstd && dy && rows > 0 && T > 1);
  // in_bwd_kernel addresses through 32-bit buffer byte offsets; larger tensors take the long-row
  // kernel (64-bit addressing), as in the forward
  const bool buf32 = rows * (long long)T < (1ll << 29);
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  int np = (T + 127) / 128;
  const int g = in_lanes(T);
  dim3 gs((unsigned)((rows * g + 255) / 256));
  const bool even = T % 2 == 0 && (((uintptr_t)y | (uintptr_t)d_a | (uintptr_t)dy) & 7) == 0;
#define MST_IN(NP_, G_, GR)                                                                            \
  do {                                                                                                 \
    if (even) hipLaunchKernelGGL((in_bwd_kernel<NP_, G_, true>), GR, block, 0, st, y, mean, rstd, rows, T, slope, d_a, d_pool0, d_pool1, dy, rowsum); \
    else hipLaunchKernelGGL((in_bwd_kernel<NP_, G_, false>), GR, block, 0, st, y, mean, rstd, rows, T, slope, d_a, d_pool0, d_pool1, dy, rowsum); \
  } while (0)
  if (buf32 && np <= 1 && g < 64) {
    if (g == 4) MST_IN(1, 4, gs);
    else if (g == 8) MST_IN(1, 8, gs);
    else if (g == 16) MST_IN(1, 16, gs);
    else MST_IN(1, 32, gs);
  } else if (buf32 && np <= 1) MST_IN(1, 64, grid);
  else if (buf32 && np <= 2) MST_IN(2, 64, grid);
  else if (buf32 && np <= 4) MST_IN(4, 64, grid);
  else if (buf32 && np <= 8) MST_IN(8, 64, grid);
#undef MST_IN
  else hipLaunchKernelGGL(in_bwd_long_kernel, grid, block, 0, st, y, mean, rstd, rows, T, slope, d_a, d_pool0, d_pool1, dy, rowsum);
  MST_CHECK_LAUNCH();
  return MST_OK;
}

int mst_bias_grad_f32(const float* dy, int32_t B, int32_t C, int32_t T, float scale, float* db,
                      int32_t accumulate, void* stream) {
  MST_REQUIRE(dy && db && B > 0 && C > 0 && T > 0 && (long long)B * T < (1ll << 30));
  hipLaunchKernelGGL(bias_grad_kernel, dim3(C), dim3(256), 0, (hipStream_t)stream, dy, B, C, T, scale,
                     db, accumulate);
  MST_CHECK_LAUNCH();
  return MST_OK;
}

int mst_bias_grad_rows_f32(const float* rowsum, int32_t B, int32_t C, float scale, float* db,
                           int32_t accumulate, void* stream) {
  MST_REQUIRE(rowsum && db && B > 0 && C > 0);
  hipLaunchKernelGGL(bias_rows_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     rowsum, B, C, scale, db, accumulate);
  MST_CHECK_LAUNCH();
  return MST_OK;
}

size_t mst_l1_workspace_size(int64_t n) { return (size_t)grid_for(n, 256 * 8, 1024) * sizeof(double); }

static int loss_launch(int mode, const float* x, const float* t, int64_t n, float* loss, void* ws,
                       void* stream) {
  MST_REQUIRE(x && t && loss && ws && n > 0);
  hipStream_t st = (hipStream_t)stream;
  int nb = grid_for(n, 256 * 8, 1024);
  double* part = (double*)ws;
  if (mode == 1) hipLaunchKernelGGL(loss_partial_kernel<1>, dim3(nb), dim3(256), 0, st, x, t, n, part);
  else hipLaunchKernelGGL(loss_partial_kernel<2>, dim3(nb), dim3(256), 0, st, x, t, n, part);
  MST_CHECK_LAUNCH();
  hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(256), 0, st, part, nb, (long long)n, loss);
  MST_CHECK_LAUNCH();
  return MST_OK;
}

int mst_l1_fwd_f32(const float* pred, const float* target, int64_t n, float* loss, void* ws,
                   void* stream) {
  return loss_launch(1, pred, target, n, loss, ws, stream);
}
int mst_mse_fwd_f32(const float* pred, const float* target, int64_t n, float* loss, void* ws,
                    void* stream) {
  return loss_launch(2, pred, target, n, loss, ws, stream);
}

int mst_l1_bwd_f32(const float* pred, const float* target, int64_t n, const float* gscale, float* dx,
                   void* stream) {
  MST_REQUIRE(pred && target && dx && n > 0);
  hipLaunchKernelGGL(l1_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, pred,
                     target, (long long)n, gscale, dx);
  MST_CHECK_LAUNCH();
  return MST_OK;
}

int mst_lrelu_bwd_f32(const float* dy, const float* y, int64_t n, float slope, float* dx,
                      void* stream) {
  MST_REQUIRE(dy && y && dx && n > 0);
  hipLaunchKernelGGL(lrelu_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, dy, y,
                     (long long)n, slope, dx);
  MST_CHECK_LAUNCH();
  return MST_OK;
}

int mst_relu_gate_bwd_f32(const float* d, const float* h, int64_t n, float s, float* out,
                          void* stream) {
  MST_REQUIRE(d && h && out && n > 0);
  hipLaunchKernelGGL(relu_gate_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, d,
                     h, (long long)n, s, out);
  MST_CHECK_LAUNCH();
  return MST_OK;
}

int mst_adam_ex_f32(float* p, const float* g, float* m, float* v, int64_t n, float lr_step,
                    float b2, float one_minus_b1, float one_minus_b2, float eps, float bc2_sqrt,
                    int32_t max_blocks, void* stream) {
  MST_REQUIRE(p && g && m && v && n > 0 && max_blocks > 0);
  MST_REQUIRE(((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16 == 0);
  launch_adam(dim3(grid_for(n / 4 + 1, 256, max_blocks)), (hipStream_t)stream, p, g, m, v,
              (long long)n, lr_step, b2, one_minus_b1, one_minus_b2, eps, bc2_sqrt, nullptr);
  MST_CHECK_LAUNCH();
  return MST_OK;
}

int mst_adam_dev_f32(float* p, const float* g, float* m, float* v, int64_t n, const float* hyper,
                     float b2, float one_minus_b1, float one_minus_b2, float eps, void* stream) {
  MST_REQUIRE(p && g && m && v && hyper && n > 0);
  MST_REQUIRE(((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16 == 0);
  launch_adam(dim3(grid_for(n / 4 + 1, 256, adam_cfg().blocks)), (hipStream_t)stream, p, g, m, v,
              (long long)n, 0.f, b2, one_minus_b1, one_minus_b2, eps, 1.f, hyper);
  MST_CHECK_LAUNCH();
  return MST_OK;
}

int mst_adam_f32(float* p, const float* g, float* m, float* v, int64_t n, float lr_step, float b2,
                 float one_minus_b1, float one_minus_b2, float eps, float bc2_sqrt, void* stream) {
  return mst_adam_ex_f32(p, g, m, v, n, lr_step, b2, one_minus_b1, one_minus_b2, eps, bc2_sqrt,
                         adam_cfg().blocks, stream);
}

int mst_scale_f32(float* x, int64_t n, float s, void* stream) {
  MST_REQUIRE(x && n >= 0);
  if (n == 0) return MST_OK;
  hipLaunchKernelGGL(scale_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x,
                     (long long)n, s);
  MST_CHECK_LAUNCH();
  return MST_OK;
}

int mst_fill_f32(float* x, int64_t n, float v, void* stream) {
  MST_REQUIRE(x && n >= 0);
  if (n == 0) return MST_OK;
  hipLaunchKernelGGL(fill_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x,
                     (long long)n, v);
  MST_CHECK_LAUNCH();
  return MST_OK;
}

int mst_onoff_f32(const float* roll, int32_t B, int32_t T, float* bin, float* onoff, void* stream) {
  MST_REQUIRE(roll && bin && onoff && B > 0 && T > 0);
  hipLaunchKernelGGL(onoff_kernel, dim3(grid_for((long long)B * T * 128)), dim3(256), 0,
                     (hipStream_t)stream, roll, B, T, bin, onoff);
  MST_CHECK_LAUNCH();
  return MST_OK;
}

const char* mst_version(void) { return "libmst_hip 0.1 gfx950"; }

int mst_device_arch(char* buf, int32_t n) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return -(int)e;
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, dev);
  if (e != hipSuccess) return -(int)e;
  int i = 0;
  for (; i + 1 < n && prop.gcnArchName[i]; ++i) buf[i] = prop.gcnArchName[i];
  if (n > 0) buf[i] = 0;
  return MST_OK;
}

}  // extern "C"
