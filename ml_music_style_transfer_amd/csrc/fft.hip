// Spectral front end on gfx950: STFT (log-power / power / mel / complex), iSTFT and
// Griffin-Lim for n_fft = 2048 (the reference's only FFT size: preprocess.py:25,48;
// inference.py:105-110; test_griffinlim.py:23).
//
// FFT design: a real 2048-point frame is packed as a 1024-point complex signal
// z[n] = x[2n] + i x[2n+1] (window applied on load). One wave owns one frame; each lane
// holds 16 complex values and the 1024-point FFT runs as radix-16 (registers) ->
// LDS transpose -> radix-16 (registers) -> LDS transpose -> radix-4, then the real-FFT
// post-twist (X[k] from Z[k], Z[1024-k]) produces the 1025 bins. Row strides of the LDS
// images are padded (68 complex); PMC showed this layout is NOT conflict-free (13.5 % of its
// LDS cycles were bank conflicts, profiles/r01/pmc_stft_frontend.txt): the frequency-major
// kernels below use fft1024_v2 instead (0 conflicts, profiles/r02). This round-1 path remains for
// the frame-major complex STFT (Griffin-Lim) and the iSTFT. Twiddles come from a 512-entry quarter-wave LDS table
// (W^(512q + r) = (-i)^q W^r), built in double precision on the host side of the
// compiler (constexpr tables, copied to LDS per workgroup).
//
// STFT workgroups: 512 threads (8 waves) x 32 frames of one clip. Results are staged
// through LDS (reusing the FFT scratch) so each (bin, 32 frames) row of the (B, F, T)
// output is written as one 128-byte run.
#include <cstdlib>

#include "common.h"
#include "mss_args.h"

namespace {

constexpr int NFFT = 2048;
constexpr int NC = 1024;        // complex FFT length
constexpr int NB = NC + 1;      // output bins
constexpr int RS = 68;          // padded LDS row stride (complex) for the 16 x 64 images
constexpr int SCR = 16 * RS;    // complex per wave scratch (1088)
constexpr int WAVES = 8;
constexpr int FR = 32;          // frames per STFT workgroup
constexpr int QT = 512;         // quarter-wave twiddle table entries

struct c2 {
  float x, y;
};
__device__ __forceinline__ c2 mk(float x, float y) { return c2{x, y}; }
__device__ __forceinline__ c2 operator+(c2 a, c2 b) { return mk(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ c2 operator-(c2 a, c2 b) { return mk(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ c2 operator*(c2 a, float s) { return mk(a.x * s, a.y * s); }
__device__ __forceinline__ c2 cmul(c2 a, c2 b) {
  return mk(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ c2 conj(c2 a) { return mk(a.x, -a.y); }

// W_2048^k (forward: exp(-2 pi i k / 2048)); INV conjugates.
template <bool INV>
__device__ __forceinline__ c2 tw(const c2* qt, int k) {
  k &= (NFFT - 1);
  int q = k >> 9, r = k & (QT - 1);
  c2 w = qt[r];  // (cos, -sin) of 2 pi r / 2048
  c2 o;
  // multiply by (-i)^q
  if (q == 0) o = w;
  else if (q == 1) o = mk(w.y, -w.x);
  else if (q == 2) o = mk(-w.x, -w.y);
  else o = mk(-w.y, w.x);
  if (INV) o.y = -o.y;
  return o;
}

// cx_sincos_turn / kPiD: common.h
struct FftTabs {
  float2 a[15 * 64];  // a[(k1 - 1) 64 + l] = W1024^(l k1)
  float2 b[3 * 16];   // b[(q - 1) 16 + l]  = W64^(l q)
  float2 p[512];      // p[k] = W2048^k
};
constexpr FftTabs make_tabs() {
  FftTabs t{};
  double c = 0, s = 0;
  for (int k1 = 1; k1 < 16; ++k1)
    for (int l = 0; l < 64; ++l) {
      cx_sincos_turn((long long)l * k1, 1024, c, s);
      t.a[(k1 - 1) * 64 + l] = float2{(float)c, (float)-s};
    }
  for (int q = 1; q < 4; ++q)
    for (int l = 0; l < 16; ++l) {
      cx_sincos_turn((long long)l * q, 64, c, s);
      t.b[(q - 1) * 16 + l] = float2{(float)c, (float)-s};
    }
  for (int k = 0; k < 512; ++k) {
    cx_sincos_turn(k, 2048, c, s);
    t.p[k] = float2{(float)c, (float)-s};
  }
  return t;
}
__device__ constexpr FftTabs kFftTabs = make_tabs();
constexpr int TAB_F4 = (int)(sizeof(FftTabs) / 16);
// W4096^(2 l + 1) = (cos, -sin)(pi (2 l + 1) / 2048), l < 64: the window phase of the odd samples
struct EhTab {
  float2 e[64];
};
constexpr EhTab make_eh() {
  EhTab t{};
  double c = 0, s = 0;
  for (int l = 0; l < 64; ++l) {
    cx_sincos_turn(2 * l + 1, 4096, c, s);
    t.e[l] = float2{(float)c, (float)-s};
  }
  return t;
}
__device__ constexpr EhTab kEh = make_eh();

// quarter-wave table qt[r] = W2048^r, r < 512: copied from the compile-time table (no f64
// sincospi per workgroup)
__device__ void build_qtable(c2* qt) {
  for (int r = threadIdx.x; r < QT; r += blockDim.x) qt[r] = mk(kFftTabs.p[r].x, kFftTabs.p[r].y);
}

template <bool INV>
__device__ __forceinline__ void dft4(c2& a0, c2& a1, c2& a2, c2& a3) {
  c2 t0 = a0 + a2, t1 = a0 - a2, t2 = a1 + a3, t3 = a1 - a3;
  c2 it3 = mk(-t3.y, t3.x);  // i * t3
  a0 = t0 + t2;
  a2 = t0 - t2;
  if (!INV) {
    a1 = t1 - it3;
    a3 = t1 + it3;
  } else {
    a1 = t1 + it3;
    a3 = t1 - it3;
  }
}

// exp(-2 pi i j / 32), j = 0..15 (forward sign), folded to immediates.
constexpr float kW32C[16] = {1.000000000f, 0.980785280f, 0.923879533f, 0.831469612f, 0.707106781f,
                             0.555570233f, 0.382683432f, 0.195090322f, 0.000000000f, -0.195090322f,
                             -0.382683432f, -0.555570233f, -0.707106781f, -0.831469612f,
                             -0.923879533f, -0.980785280f};
constexpr float kW32S[16] = {0.000000000f, -0.195090322f, -0.382683432f, -0.555570233f,
                             -0.707106781f, -0.831469612f, -0.923879533f, -0.980785280f,
                             -1.000000000f, -0.980785280f, -0.923879533f, -0.831469612f,
                             -0.707106781f, -0.555570233f, -0.382683432f, -0.195090322f};
// v[k] *= w^k for k = 1..15, powers by a depth-4 product tree (one table lookup per pass
// instead of fifteen; error a few ulp).
__device__ __forceinline__ void twiddle_powers(c2 v[16], c2 w1) {
  const c2 w2 = cmul(w1, w1), w4 = cmul(w2, w2), w8 = cmul(w4, w4);
  const c2 w3 = cmul(w2, w1), w5 = cmul(w4, w1), w6 = cmul(w4, w2), w7 = cmul(w4, w3);
  v[1] = cmul(v[1], w1);
  v[2] = cmul(v[2], w2);
  v[3] = cmul(v[3], w3);
  v[4] = cmul(v[4], w4);
  v[5] = cmul(v[5], w5);
  v[6] = cmul(v[6], w6);
  v[7] = cmul(v[7], w7);
  v[8] = cmul(v[8], w8);
  v[9] = cmul(v[9], cmul(w8, w1));
  v[10] = cmul(v[10], cmul(w8, w2));
  v[11] = cmul(v[11], cmul(w8, w3));
  v[12] = cmul(v[12], cmul(w8, w4));
  v[13] = cmul(v[13], cmul(w8, w5));
  v[14] = cmul(v[14], cmul(w8, w6));
  v[15] = cmul(v[15], cmul(w8, w7));
}

// W16^m as compile-time constants (forward sign).
__device__ __forceinline__ c2 w16(int m) {
  constexpr float C1 = 0.92387953251128674f, S1 = 0.38268343236508978f, R2 = 0.70710678118654752f;
  switch (m & 15) {
    case 0: return mk(1.f, 0.f);
    case 1: return mk(C1, -S1);
    case 2: return mk(R2, -R2);
    case 3: return mk(S1, -C1);
    case 4: return mk(0.f, -1.f);
    case 5: return mk(-S1, -C1);
    case 6: return mk(-R2, -R2);
    case 7: return mk(-C1, -S1);
    case 8: return mk(-1.f, 0.f);
    case 9: return mk(-C1, S1);
    default: return mk(0.f, 0.f);  // not needed (j1*k2 <= 9)
  }
}

// In-register 16-point DFT: out[k] = sum_j v[j] W16^{jk} (INV: conjugate twiddles).
template <bool INV>
__device__ __forceinline__ void dft16(c2 v[16]) {
#pragma unroll
  for (int j1 = 0; j1 < 4; ++j1) dft4<INV>(v[j1], v[j1 + 4], v[j1 + 8], v[j1 + 12]);
  // v[j1 + 4 k2] = Y[j1][k2]; twiddle by W16^{j1 k2}
#pragma unroll
  for (int j1 = 1; j1 < 4; ++j1)
#pragma unroll
    for (int k2 = 1; k2 < 4; ++k2) {
      c2 w = w16(j1 * k2);
      if (INV) w.y = -w.y;
      v[j1 + 4 * k2] = cmul(v[j1 + 4 * k2], w);
    }
  // DFT4 over j1 for each k2: X[k2 + 4 k1] = sum_j1 W4^{j1 k1} Y[j1][k2]
#pragma unroll
  for (int k2 = 0; k2 < 4; ++k2) dft4<INV>(v[4 * k2], v[4 * k2 + 1], v[4 * k2 + 2], v[4 * k2 + 3]);
  // now v[j1' + 4 k2] holds X[k2 + 4 k1] with k1 = j1' -> transpose 4x4 into natural order
  c2 t[16];
#pragma unroll
  for (int k2 = 0; k2 < 4; ++k2)
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) t[k2 + 4 * k1] = v[k1 + 4 * k2];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = t[i];
}

// 1024-point complex FFT of one wave. Input v[j] = z[lane + 64 j]; on return S[k]
// (k = 0..1023, natural order, unnormalised) holds Z[k]. S: this wave's scratch.
template <bool INV>
__device__ void fft1024(c2 v[16], c2* S, const c2* qt, int lane) {
  // pass A: radix-16 over j, twiddle W1024^{lane k1} = W2048^{2 lane k1}
  dft16<INV>(v);
  twiddle_powers(v, tw<INV>(qt, 2 * lane));  // W1024^{lane k1}
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) S[k1 * RS + lane] = v[k1];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  // pass B: lane = k1*4 + lp; 16-point DFT over jp of X1[k1][lp + 4 jp]
  {
    const int k1 = lane >> 2, lp = lane & 3;
#pragma unroll
    for (int jp = 0; jp < 16; ++jp) v[jp] = S[k1 * RS + lp + 4 * jp];
    dft16<INV>(v);
    twiddle_powers(v, tw<INV>(qt, 32 * lp));  // W64^{lp mp}
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int mp = 0; mp < 16; ++mp) S[k1 * RS + mp * 4 + lp] = v[mp];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  // pass C: (k1 = lane & 15, mp = (lane >> 4) + 4 q), 4-point DFT over lp
  {
    const int k1 = lane & 15;
    c2 c[4][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int mp = (lane >> 4) + 4 * q;
#pragma unroll
      for (int lp = 0; lp < 4; ++lp) c[q][lp] = S[k1 * RS + mp * 4 + lp];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int mp = (lane >> 4) + 4 * q;
      dft4<INV>(c[q][0], c[q][1], c[q][2], c[q][3]);
#pragma unroll
      for (int m2 = 0; m2 < 4; ++m2) S[k1 + 16 * mp + 256 * m2] = c[q][m2];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ float hann_w(const c2* qt, int n) {
  // 0.5 - 0.5 cos(2 pi n / 2048), periodic Hann (scipy get_window('hann', 2048, fftbins=True))
  return 0.5f - 0.5f * tw<false>(qt, n).x;
}

// Real-FFT post-twist: X[k] for k = lane + 64 j from Z in S; X[1024] via lane 0.
__device__ __forceinline__ c2 post_bin(const c2* S, c2 wk, int k) {
  c2 A = S[k];
  c2 Bc = conj(S[(NC - k) & (NC - 1)]);
  c2 xe = (A + Bc) * 0.5f;
  c2 d = A - Bc;
  c2 xo = mk(0.5f * d.y, -0.5f * d.x);  // -i/2 * d
  return xe + cmul(wk, xo);
}

// W2048^(lane + 64 j) from e = W2048^lane.
__device__ __forceinline__ c2 tw_bin(c2 e, int j) { return cmul(e, mk(kW32C[j], kW32S[j])); }

// Periodic Hann 0.5 - 0.5 cos(2 pi m / 2048) = sin^2(pi m / 2048), in the sin^2 form so the
// small values at the frame edges keep their relative precision. For m = 2n, n = lane + 64 j:
// sin(pi m / 2048) = -Im(W2048^n) with W2048^n = e1 W32^j; for m = 2n + 1 the same with
// eh = W4096^{2 lane + 1}.
__device__ __forceinline__ float hann_sq(c2 e, int j) {
  const float s = e.x * kW32S[j] + e.y * kW32C[j];  // Im(e W32^j)
  return s * s;
}

__device__ __forceinline__ float log1p_fast(float p) {
  // log1p via log(u) * p / (u - 1) (exact-ish for tiny p), hardware log2
  float u = 1.f + p;
  float d = u - 1.f;
  float l = __log2f(u) * 0.69314718055994531f;
  return d == 0.f ? p : l * (p * __builtin_amdgcn_rcpf(d));  // 1-ulp v_rcp, not an IEEE divide
}

enum { MODE_LOGPOW = 0, MODE_POWER = 1, MODE_MEL = 2, MODE_COMPLEX = 3 };

struct MelTab {
  const int* start;
  const int* len;
  const int* woff;
  const float* w;
  int n_mels;
};

// Raw (unwindowed) samples of frame f for z[lane + 64 j] (center padding: reflect or zeros).
__device__ __forceinline__ void fetch_frame(const float* xr, int L, int f, int hop, int pad_mode,
                                            int lane, float2 raw[16]) {
  const int s0 = f * hop - NFFT / 2;
  const bool interior = s0 >= 0 && s0 + NFFT <= L && ((((uintptr_t)(xr + s0)) & 7) == 0);
  if (interior) {
    const float2* p = reinterpret_cast<const float2*>(xr + s0);
#pragma unroll
    for (int j = 0; j < 16; ++j) raw[j] = p[lane + 64 * j];
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int n = lane + 64 * j;
      float e[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        int s = s0 + 2 * n + h;
        float val;
        if (s >= 0 && s < L) val = xr[s];
        else if (pad_mode == MST_PAD_CONSTANT) val = 0.f;
        else {
          if (s < 0) s = -s;
          if (s >= L) s = 2 * (L - 1) - s;
          val = (s >= 0 && s < L) ? xr[s] : 0.f;
        }
        e[h] = val;
      }
      raw[j] = make_float2(e[0], e[1]);
    }
  }
}

// STFT: 512 threads = 8 waves, 32 frames per workgroup in 4 rounds of 8 (one frame per wave).
// Twiddles and window values come from one per-lane table lookup times compile-time roots of
// unity (see twiddle_powers / tw_bin / hann_sq); each wave leaves its frame's 1025 results in its own LDS scratch (offset by
// 8 floats per wave so the transposed read is bank-conflict-free), and after a barrier the
// workgroup writes the round as (bin, 8 frames) runs of the frequency-major (B, F, T) output.
// 73.7 KB LDS per workgroup.
template <int MODE>
__global__ __launch_bounds__(512, 4) void stft_kernel(const float* __restrict__ x, int L, int T,
                                                      int hop, int pad_mode,
                                                      float* __restrict__ out, MelTab mel) {
  __shared__ __attribute__((aligned(16))) c2 scratch[WAVES * SCR];
  __shared__ c2 qt[QT];
  __shared__ c2 eht[64];  // W4096^{2 lane + 1}: window phase of the odd samples
  const int b = blockIdx.y;
  const int f0 = blockIdx.x * FR;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  build_qtable(qt);
  if (threadIdx.x < 64) eht[threadIdx.x] = mk(kEh.e[threadIdx.x].x, kEh.e[threadIdx.x].y);
  __syncthreads();
  const float* xr = x + (long long)b * L;
  c2* S = scratch + wave * SCR;
  float* Sf = reinterpret_cast<float*>(scratch);
  constexpr int SCRF = 2 * SCR;           // floats per wave scratch
  float* P = Sf + wave * SCRF + 8 * wave;  // this wave's staged results
  constexpr int MEL_OFF = 1200;
  const int nfr = min(FR, T - f0);
  // float4 row stores need 16-byte aligned (bin, frame 8r) addresses: T % 4 == 0
  const bool vec4 = (T & 3) == 0 && ((uintptr_t)out & 15) == 0;

#pragma unroll 1
  for (int r = 0; r < FR / WAVES; ++r) {
    const int fl = WAVES * r + wave;
    const int f = f0 + fl;
    if (fl < nfr) {
      c2 v[16];
      {
        float2 raw[16];
        fetch_frame(xr, L, f, hop, pad_mode, lane, raw);
        const c2 e1 = tw<false>(qt, lane), eh = eht[lane];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = mk(raw[j].x * hann_sq(e1, j), raw[j].y * hann_sq(eh, j));
      }
      fft1024<false>(v, S, qt, lane);
      const c2 e1 = tw<false>(qt, lane);  // W2048^lane
      if (MODE == MODE_COMPLEX) {
        float2* o = reinterpret_cast<float2*>(out) + ((long long)b * T + f) * NB;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int k = lane + 64 * j;
          const c2 X = post_bin(S, tw_bin(e1, j), k);
          o[k] = make_float2(X.x, X.y);
        }
        if (lane == 0) {
          const c2 z0 = S[0];
          o[NC] = make_float2(z0.x - z0.y, 0.f);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
      } else {
        float pw[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const c2 X = post_bin(S, tw_bin(e1, j), lane + 64 * j);
          pw[j] = X.x * X.x + X.y * X.y;
        }
        const c2 z0 = S[0];
        const float xn = z0.x - z0.y;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < 16; ++j)
          P[lane + 64 * j] = (MODE == MODE_LOGPOW) ? log1p_fast(pw[j]) : pw[j];
        if (lane == 0) P[NC] = (MODE == MODE_LOGPOW) ? log1p_fast(xn * xn) : xn * xn;
        if (MODE == MODE_MEL) {
          // mel bands from the power spectrum (P holds power in MEL mode)
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int m = lane + 64 * h;
            float acc = 0.f;
            if (m < mel.n_mels) {
              const int st = mel.start[m], n = mel.len[m], wo = mel.woff[m];
              for (int q = 0; q < n; ++q) acc += mel.w[wo + q] * P[st + q];
            }
            P[MEL_OFF + m] = acc;
          }
        }
      }
    }
    if (MODE == MODE_COMPLEX) continue;
    __syncthreads();
    // write round r: frames f0 + 8r .. +7, as (row, 8 frames) runs
    const int nr = MODE == MODE_MEL ? mel.n_mels : NB;
    const int roff = MODE == MODE_MEL ? MEL_OFF : 0;
    const int nfr_r = min(WAVES, nfr - WAVES * r);
    float* ob = out + (long long)b * nr * T + f0 + WAVES * r;
    if (vec4) {
      // two float4 stores per row (frames 0-3, 4-7 of the round): 4x fewer store
      // instructions than one 4-byte store per frame (the write phase is store-issue bound)
      for (int e = threadIdx.x; e < nr * 2; e += blockDim.x) {
        const int k = e >> 1, w0 = 4 * (e & 1);
        float* o = ob + (long long)k * T + w0;
        const float* src = Sf + w0 * (SCRF + 8) + roff + k;
        if (w0 + 3 < nfr_r) {
          *reinterpret_cast<float4*>(o) = make_float4(src[0], src[SCRF + 8], src[2 * (SCRF + 8)],
                                                      src[3 * (SCRF + 8)]);
        } else {
          for (int w = 0; w < 4 && w0 + w < nfr_r; ++w) o[w] = src[w * (SCRF + 8)];
        }
      }
    } else {
      for (int e = threadIdx.x; e < nr * WAVES; e += blockDim.x) {
        const int k = e >> 3, w = e & 7;
        if (w < nfr_r) ob[(long long)k * T + w] = Sf[w * SCRF + 8 * w + roff + k];
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Frequency-major STFT (log-power / power / mel), the (B, F, T) layout of
// process_spectrum_from_chunk (preprocess.py:47-49) and melspectrogram (plot_spec.py:20).
//
// Output. The round-1 kernel's (bin, 8 frames) 32-byte row pieces, written by one workgroup in
// four rounds, cost ~90 of its 238 us for config 2 (profiles/r02/
// stft_ablation_and_store_patterns.txt). The same bytes written as 64-byte pieces by
// workgroups that all belong to ONE clip and share one XCD (its L2 merges the pieces of every
// line before they reach HBM) run as fast as a contiguous write (38 us, 6.9 TB/s). So a
// workgroup owns 16 consecutive frames of one clip, and workgroup g serves clip
// (g / (8 nblk)) * 8 + g % 8 (g % 8 is the XCD group label), frames 16 ((g / 8) % nblk) + ...
// Wave w computes frames w and 8 + w (the first one's results wait in registers); then the 16
// frames go to LDS [frame][bin] and leave as (bin, 16 frames) rows, four float4 per bin.
//
// FFT (per wave, one frame): z[n] = x[2n] + i x[2n+1] windowed, n = l + 64 j (lane l, register
// j), 1024 = 16 x 4 x 16:
//   A  DFT16 over j in registers, twiddle W1024^(l k1) (LDS table);
//   B1 DFT4 over the lane bits 4-5: two v_permlane{32,16}_swap stages exchange those lane bits
//      with register bits 3-2 (no LDS), DFT4 in registers, twiddle W64^(l_lo q_lo);
//   B2 one LDS transpose (XOR-swizzled, conflict-free both ways), DFT16 in registers: lane t
//      ends with Z[t + 64 j] in register j.
// The real-FFT post-twist pairs bin k = l + 64 j with 1024 - k, whose Z sits in lane 64 - l,
// register 15 - j: 16 ds_bpermute (no LDS memory), one table twiddle per pair. One LDS round
// trip per frame instead of three, twiddles from tables instead of product trees, and
// log1p(p) = log(1 + p) on the hardware log (absolute error <= 1e-6, inside the 1e-4 bar).
// ---------------------------------------------------------------------------
#ifndef FM_WAVES
#define FM_WAVES 8                 // frequency-major STFT: waves per workgroup (8 or 16), mel / complex
#endif
#ifndef FM_WAVES_POW
#define FM_WAVES_POW 16            // ... for log-power / power
#endif
constexpr int RSTR_MEL = 130;      // staging row stride for <= 128 mel bands (= 2 mod 32)


__device__ __forceinline__ void swap32(c2& lo, c2& hi) {  // lane bit 5 <-> the lo/hi pair
  auto rx = __builtin_amdgcn_permlane32_swap(__float_as_uint(lo.x), __float_as_uint(hi.x), false, false);
  auto ry = __builtin_amdgcn_permlane32_swap(__float_as_uint(lo.y), __float_as_uint(hi.y), false, false);
  lo = mk(__uint_as_float(rx[0]), __uint_as_float(ry[0]));
  hi = mk(__uint_as_float(rx[1]), __uint_as_float(ry[1]));
}
__device__ __forceinline__ void swap16(c2& lo, c2& hi) {  // lane bit 4 <-> the lo/hi pair
  auto rx = __builtin_amdgcn_permlane16_swap(__float_as_uint(lo.x), __float_as_uint(hi.x), false, false);
  auto ry = __builtin_amdgcn_permlane16_swap(__float_as_uint(lo.y), __float_as_uint(hi.y), false, false);
  lo = mk(__uint_as_float(rx[0]), __uint_as_float(ry[0]));
  hi = mk(__uint_as_float(rx[1]), __uint_as_float(ry[1]));
}

// Forward 1024-point FFT of one wave: v[j] = z[lane + 64 j] in, v[j] = Z[lane + 64 j] out.
// S: this wave's 1024-entry LDS scratch; tabs: the LDS copy of kFftTabs.
__device__ __forceinline__ void fft1024_v2(c2 v[16], c2* S, const FftTabs& tb, int lane) {
  dft16<false>(v);  // Y[l][k1] in v[k1]
#pragma unroll
  for (int k1 = 1; k1 < 16; ++k1) {
    const float2 w = tb.a[(k1 - 1) * 64 + lane];
    v[k1] = cmul(v[k1], mk(w.x, w.y));
  }
  // B1: lane bits (5, 4) <-> register bits (3, 2): lane (l_lo, k1 >> 2), register a + 4 l_hi
#pragma unroll
  for (int r = 0; r < 8; ++r) swap32(v[r], v[r + 8]);
#pragma unroll
  for (int r = 0; r < 16; ++r)
    if ((r & 4) == 0) swap16(v[r], v[r + 4]);
#pragma unroll
  for (int a = 0; a < 4; ++a) dft4<false>(v[a], v[a + 4], v[a + 8], v[a + 12]);  // -> q_lo
  const int llo = lane & 15, c = lane >> 4;
#pragma unroll
  for (int q = 1; q < 4; ++q) {
    const float2 w = tb.b[(q - 1) * 16 + llo];
#pragma unroll
    for (int a = 0; a < 4; ++a) v[a + 4 * q] = cmul(v[a + 4 * q], mk(w.x, w.y));
  }
  // B2: pair p = k1 + 16 q_lo (k1 = a + 4 c) gathers its 16 l_lo values in lane p. Pairs are
  // 17 entries apart: the writes (16 lanes per pair) and the reads (lane t, entry i) are
  // bank-conflict-free, and every address is a per-lane base plus an immediate offset.
  c2* Sw = S + 68 * c + llo;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int a = 0; a < 4; ++a) Sw[17 * (a + 16 * q)] = v[a + 4 * q];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const c2* Sr = S + 17 * lane;
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = Sr[i];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  dft16<false>(v);  // Z[lane + 64 q_hi] in v[q_hi]
}


// fft1024_v2 with the twiddles formed from two values: w1 = W1024^lane (stage A, powers by
// twiddle_powers' depth-4 product tree) and wb = W64^(lane & 15) (stage B1, wb^2, wb^3): a
// caller that keeps no table in LDS issues two loads early instead of eighteen on the FFT's
// critical path (error: a few ulp per twiddle).
__device__ __forceinline__ void fft1024_v2p(c2 v[16], c2* S, c2 w1, c2 wb, int lane) {
  dft16<false>(v);
  twiddle_powers(v, w1);
#pragma unroll
  for (int r = 0; r < 8; ++r) swap32(v[r], v[r + 8]);
#pragma unroll
  for (int r = 0; r < 16; ++r)
    if ((r & 4) == 0) swap16(v[r], v[r + 4]);
#pragma unroll
  for (int a = 0; a < 4; ++a) dft4<false>(v[a], v[a + 4], v[a + 8], v[a + 12]);
  const int llo = lane & 15, c = lane >> 4;
  const c2 wb2 = cmul(wb, wb), wb3 = cmul(wb2, wb);
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    v[a + 4] = cmul(v[a + 4], wb);
    v[a + 8] = cmul(v[a + 8], wb2);
    v[a + 12] = cmul(v[a + 12], wb3);
  }
  c2* Sw = S + 68 * c + llo;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int a = 0; a < 4; ++a) Sw[17 * (a + 16 * q)] = v[a + 4 * q];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const c2* Sr = S + 17 * lane;
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = Sr[i];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  dft16<false>(v);
}

__device__ __forceinline__ float bperm(int src_byte, float x) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(src_byte, __float_as_int(x)));
}

__device__ __forceinline__ float ln_1p_quarter(float p4) {  // log1p(p4 / 4)
  return __log2f(fmaf(0.25f, p4, 1.f)) * 0.69314718055994531f;
}

// Power spectrum from Z[lane + 64 j] in v, as bin pairs: r[2j] = bin l + 64 j, r[2j + 1] =
// bin 1024 - l - 64 j (j = 0..7), r[16] = bin 512 (meaningful in lane 0); LOG: log1p(power).
// 2 X[k] = E + W^k D, 2 conj(X[1024 - k]) = E - W^k D with E = Z[k] + conj(Z[1024 - k]),
// D = -i (Z[k] - conj(Z[1024 - k])); Z[1024 - k] lives in lane 64 - l, register 15 - j.
template <bool LOG>
__device__ __forceinline__ void power_pairs_v2(const c2 v[16], const FftTabs& tb, int lane,
                                               float r[17]) {
  const int src = ((64 - lane) & 63) * 4;
  c2 prev = v[0];  // lane 0's partner 1024 - 64 j is its own v[16 - j] (v[0] for j = 0)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const c2 bpj = mk(bperm(src, v[15 - j].x), bperm(src, v[15 - j].y));
    const c2 Bq = lane == 0 ? prev : bpj;
    prev = bpj;
    const c2 A = v[j];
    const c2 E = mk(A.x + Bq.x, A.y - Bq.y);
    const c2 D = mk(A.y + Bq.y, Bq.x - A.x);  // -i (A - conj(Bq))
    const float2 w = tb.p[lane + 64 * j];
    const c2 TD = cmul(mk(w.x, w.y), D);
    const c2 P = E + TD, M = E - TD;
    const float p4 = P.x * P.x + P.y * P.y, m4 = M.x * M.x + M.y * M.y;
    r[2 * j] = LOG ? ln_1p_quarter(p4) : 0.25f * p4;
    r[2 * j + 1] = LOG ? ln_1p_quarter(m4) : 0.25f * m4;
  }
  const float z4 = 4.f * (v[8].x * v[8].x + v[8].y * v[8].y);
  r[16] = LOG ? ln_1p_quarter(z4) : 0.25f * z4;
}

// Complex bins from Z[lane + 64 j] in v, in power_pairs_v2's pairing: x[2j] = X[l + 64 j],
// x[2j + 1] = X[1024 - l - 64 j] (j = 0..7; lane 0, j = 0: X[1024]), x[16] = X[512] (lane 0).
__device__ __forceinline__ void complex_pairs_v2(const c2 v[16], const FftTabs& tb, int lane,
                                                 c2 x[17]) {
  const int src = ((64 - lane) & 63) * 4;
  c2 prev = v[0];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const c2 bpj = mk(bperm(src, v[15 - j].x), bperm(src, v[15 - j].y));
    const c2 Bq = lane == 0 ? prev : bpj;
    prev = bpj;
    const c2 A = v[j];
    const c2 E = mk(A.x + Bq.x, A.y - Bq.y);
    const c2 D = mk(A.y + Bq.y, Bq.x - A.x);
    const float2 w = tb.p[lane + 64 * j];
    const c2 TD = cmul(mk(w.x, w.y), D);
    const c2 P = E + TD, M = E - TD;  // 2 X[k], 2 conj X[1024 - k]
    x[2 * j] = mk(0.5f * P.x, 0.5f * P.y);
    x[2 * j + 1] = mk(0.5f * M.x, -0.5f * M.y);
  }
  x[16] = mk(v[8].x, -v[8].y);  // X[512] = conj Z[512]
}

// staging position of (frame row, bin k < 1024): row stride 1024, bits of k XORed with the row's
// quad index so the write-out's 4-row column gathers are bank-conflict-free (16 rows: 8 bins x
// 4 quads per 32 lanes, XOR 8 q; 8 rows: 16 bins x 2 quads, XOR 16 q)
template <int ROWS>
__device__ __forceinline__ int stage_pos(int row, int k) {
  return row * 1024 + (k ^ ((ROWS == 16 ? 8 : 16) * ((row >> 2) & (ROWS / 4 - 1))));
}

// Raw samples of frame f as z[lane + 64 j] = (x_pad[s0 + 2n], x_pad[s0 + 2n + 1]), n = lane + 64 j,
// s0 = f hop - 1024, center padding reflect or zeros. Exactly 16 buffer loads on every path and
// no use of the loaded data here (the callers' vmcnt accounting depends on both): a frame that
// touches the padding loads per-lane pairs and records what fix_frame must do with them. A
// reflected pair is an adjacent pair read backwards: x_pad[s] = x[-s] (s < 0) and
// x[2 L - 2 - s] (s >= L), so (x_pad[s], x_pad[s + 1]) is the pair at -s - 1 or at
// 2 L - 3 - s, swapped; zero padding loads the clamped pair and drops the outside halves.
struct FrameFix {
  unsigned swap;  // bit j: swap pair j (reflect)
  unsigned zlo;   // bit j: pair j's first sample is padding (zeros)
  unsigned zhi;   // bit j: its second sample is padding
  unsigned sel;   // bit j: the wanted first sample is the loaded pair's second (zeros, clamped)
  int edge;       // wave-uniform: the frame touches the padding
};

__device__ __forceinline__ void fetch_frame16(const float* xr, int L, int f, int hop, int pad_mode,
                                              int lane, float2 raw[16], FrameFix& fx) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xr), (short)0, L * 4, 0x00020000);
  const int s0 = f * hop - NFFT / 2;
  fx.edge = !(s0 >= 0 && s0 + NFFT <= L);
  fx.swap = fx.zlo = fx.zhi = fx.sel = 0;
  if (!fx.edge) {
#pragma unroll
    for (int j = 0; j < 16; ++j)
      raw[j] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rs, 8 * lane, 4 * s0 + 512 * j, 0));
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int s = s0 + 2 * (lane + 64 * j);
      int a;
      if (pad_mode == MST_PAD_REFLECT) {
        const bool left = s < 0, right = s + 1 >= L;
        a = left ? -s - 1 : (right ? 2 * L - 3 - s : s);
        fx.swap |= (unsigned)(left || right) << j;
      } else {
        a = min(max(s, 0), L - 2);
        fx.zlo |= (unsigned)(s < 0 || s >= L) << j;
        fx.zhi |= (unsigned)(s + 1 < 0 || s + 1 >= L) << j;
        fx.sel |= (unsigned)(s == a + 1) << j;  // only at the right end: (x[L-1], 0)
      }
      raw[j] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rs, 4 * a, 0, 0));
    }
  }
}

__device__ __forceinline__ void fix_frame(float2 raw[16], const FrameFix& fx) {
  if (!fx.edge) return;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const float2 p = raw[j];
    float lo = ((fx.swap | fx.sel) >> j) & 1 ? p.y : p.x;
    float hi = (fx.swap >> j) & 1 ? p.x : p.y;
    if ((fx.zlo >> j) & 1) lo = 0.f;
    if ((fx.zhi >> j) & 1) hi = 0.f;
    raw[j] = make_float2(lo, hi);
  }
}

// Persistent workgroups, one per CU: 16 waves, one frame each per 16-frame block. WG g serves
// XCD group x = g % 8, i.e. clips x, x + 8, ..., walking that group's (clip, block) list with
// stride W (WGs per group): at any moment a group's WGs work on a few whole clips, whose row
// pieces the group's L2 merges.
//
// Input: a block's 16 frames span (15 hop + 2048) samples (23.5 KB at hop 256) but fetching
// every frame separately moves 128 KB through the load path, 8x over; the round-2 stamps
// (tools/micro/stft_stamps.hip) had the per-wave prefetch issue alone at ~4.9k cycles per
// block. So the next block's span is DMA'd into LDS (buffer_load ... lds, 1 KB per
// instruction, out-of-range reads give the zero padding, per-sample sources the reflect
// padding) during the staging phase, into the scratch half the staging does not use, and each
// wave reads its frame from there at the start of the block.
//
// Stores and loads (LDS-DMA included) share vmcnt and complete in issue order, so the DMA is
// issued before the write-out, the write-out is a fixed count NST of buffer stores (dropped
// out-of-range offsets instead of branches), the loop entry issues NST dropped stores too, and
// the top of the loop waits vmcnt(NST): its own DMA has landed, the previous block's stores
// stay in flight. Barriers are raw s_barrier + lgkmcnt(0): __syncthreads() would drain vmcnt.
// FMW (template): waves per workgroup = frames per block, 16 (one workgroup per CU) or 8 (two)
#ifdef STFT_STAMPS  // dev instrumentation (tools/micro/stft_stamps.hip)
__device__ unsigned long long g_stamps[512 * 16 * 16 * 16];
#define STAMP(i) do { if (lane == 0 && blockIdx.x < 512 && it < 16) \
    g_stamps[((blockIdx.x * 16 + (threadIdx.x >> 6)) * 16 + it) * 16 + (i)] = clock64(); } while (0)
#else
#define STAMP(i) do { } while (0)
#endif
#define LDS_BARRIER() do { __builtin_amdgcn_s_waitcnt(0xc07f); __builtin_amdgcn_s_barrier(); } while (0)

// LDS-DMA in inline asm (cdna_hip_programming.md 5.7): hipcc does not model the asm, so it neither
// counts it nor drains it before later LDS accesses (as a builtin DMA it would insert vmcnt(0)
// before every LDS access that may alias, waiting for the write-out's stores as well); the
// kernel waits for it itself (vmcnt(NST), then a barrier, then the reads). M0 is written and
// restored inside the statement.
__device__ __forceinline__ void dma_b128(__amdgpu_buffer_rsrc_t rs, unsigned lds_addr, int voff, int soff) {
  unsigned keep;
  asm volatile(
      "s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rs), "s"(lds_addr), "s"(soff)
      : "memory");
}
__device__ __forceinline__ void dma_b32(__amdgpu_buffer_rsrc_t rs, unsigned lds_addr, int voff) {
  unsigned keep;
  asm volatile(
      "s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dword %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rs), "s"(lds_addr)
      : "memory");
}

// DMA the span of a block (samples s_lo .. s_lo + sp of clip xr, padded) into LDS span[], spread
// over the workgroup's waves. Interior blocks with a 16-byte aligned start move 16 B per lane;
// the others one sample per lane from its own source (reflect), or from out of range (zeros).
template <int FMW>
__device__ __forceinline__ void load_span(const float* xr, int L, int s_lo, int sp, int pad_mode,
                                          float* span, int wave, int lane) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xr), (short)0, L * 4, 0x00020000);
  const unsigned base = (unsigned)(uintptr_t)span;  // LDS byte address (low half of the flat one)
  const bool fast = s_lo >= 0 && s_lo + sp <= L && ((((uintptr_t)(xr + s_lo)) & 15) == 0);
  if (fast) {
    for (int i = wave; i * 256 < sp; i += FMW)
      dma_b128(rs, __builtin_amdgcn_readfirstlane(base + 1024 * i), 16 * lane,
               __builtin_amdgcn_readfirstlane(4 * s_lo + 1024 * i));
  } else {
    for (int i = wave; i * 64 < sp; i += FMW) {
      const int s = s_lo + 64 * i + lane;
      int src;
      if (pad_mode == MST_PAD_REFLECT) src = s < 0 ? -s : (s >= L ? 2 * (L - 1) - s : s);
      else src = (s < 0 || s >= L) ? L : s;  // L: out of range, reads 0
      dma_b32(rs, __builtin_amdgcn_readfirstlane(base + 256 * i), 4 * src);
    }
  }
}

template <int MODE, bool V4, int FMW>
__global__ __launch_bounds__(64 * FMW, 4) void stft_fm_kernel(const float* __restrict__ x, int B,
                                                               int L, int T, int hop, int pad_mode,
                                                               float* __restrict__ out, MelTab mel,
                                                               int W) {
  // FMW x 8,704 B scratch + 12,160 B of tables: 151,424 B (16 waves, one workgroup per CU) or
  // 81,792 B (8 waves, two per CU)
  __shared__ __attribute__((aligned(16))) c2 scratch[FMW * SCR];
  __shared__ __attribute__((aligned(16))) FftTabs tb;
  constexpr int FPB = FMW;                // frames per block
  constexpr int SPAN_OFF = FPB * NC * 4;  // bytes: the span sits after the staging rows
  const int nblk = (T + FPB - 1) / FPB;
  const int xg = blockIdx.x & 7, wi = blockIdx.x >> 3;
  const int U = (B - xg + 7) / 8 * nblk;  // blocks of this XCD group
  if (wi >= U) return;                    // whole workgroup: before any barrier
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  {
    const float4* src = reinterpret_cast<const float4*>(&kFftTabs);
    float4* dst = reinterpret_cast<float4*>(&tb);
    for (int i = threadIdx.x; i < TAB_F4; i += blockDim.x) dst[i] = src[i];
  }
  c2* S = scratch + wave * SCR;
  float* Sf = reinterpret_cast<float*>(scratch);
  float* span = reinterpret_cast<float*>(reinterpret_cast<char*>(scratch) + SPAN_OFF);
  const int sp = (FPB - 1) * hop + NFFT;  // span samples (launcher: fits after the staging)
  constexpr bool MELM = MODE == MODE_MEL;
  constexpr bool CPLX = MODE == MODE_COMPLEX;  // frame-major (B, T, F, 2): stored from registers
  const int nrows = MELM ? mel.n_mels : NB;
  const int clip_bytes = CPLX ? NB * T * 8 : nrows * T * 4;  // < 2^31: checked by the launcher
  // this lane's 32 window weights (Hann at samples 2n, 2n + 1, n = lane + 64 j), kept in
  // registers for the whole kernel (80 -> 112 VGPRs, still 4 waves per SIMD): 32 multiplies
  // per frame instead of ~110 instructions recomputing them
  float wwe[16], wwo[16];
  {
    const int lane = threadIdx.x & 63;
    double sn, cs;
    sincospi((2.0 * lane) / 2048.0, &sn, &cs);
    const c2 e1 = mk((float)cs, (float)-sn);
    sincospi((2.0 * lane + 1.0) / 2048.0, &sn, &cs);
    const c2 eh = mk((float)cs, (float)-sn);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      wwe[j] = hann_sq(e1, j);
      wwo[j] = hann_sq(eh, j);
    }
  }
  const long long rowT = T;
  auto clip_of = [&](int u) { return xg + 8 * (u / nblk); };
  auto frame0_of = [&](int u) { return (u % nblk) * FPB; };
  constexpr int NST = CPLX ? 17 : (MELM ? 1 : 5);  // write-out stores per thread per block (V4)
  constexpr int VM_NST = 0x0f70 | (NST & 15);  // s_waitcnt vmcnt(NST), expcnt/lgkmcnt unmasked

  load_span<FMW>(x + (long long)clip_of(wi) * L, L, frame0_of(wi) * hop - NFFT / 2, sp, pad_mode, span,
            wave, threadIdx.x & 63);
  if (V4) {  // the loop body's store tail, dropped (zero-size descriptor); distinct offsets so
            // none of them is merged away: the loop-top vmcnt(NST) counts exactly NST stores
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0, 0x00020000);
#pragma unroll
    for (int i = 0; i < NST; ++i) __builtin_amdgcn_raw_buffer_store_b32(0, rs, 16 * i, 0, 0);
  }
#pragma unroll 1
  for (int u = wi, it = 0; u < U; u += W, ++it) {
    // every lane-derived value below is recomputed per block from a laundered thread index and
    // laundered window phases / table offset: hoisted out of the loop they outnumber the free
    // registers and the kernel spills
    int tid = threadIdx.x, toff = 0;
    __asm__ volatile("" : "+v"(tid), "+v"(toff));
    const FftTabs& tbl = *reinterpret_cast<const FftTabs*>(reinterpret_cast<const char*>(&tb) + toff);
    const int lane = tid & 63;
    STAMP(0);
    if (V4) __builtin_amdgcn_s_waitcnt(VM_NST);  // this wave's span DMA has landed
    else __builtin_amdgcn_s_waitcnt(0x0f70);
    LDS_BARRIER();  // every wave's DMA landed; the previous block's staging is read out
    const int b = clip_of(u), f0 = frame0_of(u);
    const int nfr = min(FPB, T - f0);
    const int fl = wave;
    float2 raw[16];
    {
      const float2* src = reinterpret_cast<const float2*>(span + fl * hop) + lane;  // hop even
#pragma unroll
      for (int j = 0; j < 16; ++j) raw[j] = src[64 * j];
    }
    LDS_BARRIER();  // the span is read: the FFT scratch may overwrite it
    STAMP(1);
    float res[17];
    c2 xc[17];  // CPLX: this lane's complex bins
    if (fl < nfr) {
      c2 v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = mk(raw[j].x * wwe[j], raw[j].y * wwo[j]);
      fft1024_v2(v, S, tbl, lane);
      if (CPLX) {
        complex_pairs_v2(v, tbl, lane, xc);
      } else if (!MELM) {
        power_pairs_v2<MODE == MODE_LOGPOW>(v, tbl, lane, res);
      } else {
        float r[17];
        power_pairs_v2<false>(v, tbl, lane, r);
        // power spectrum into this wave's scratch (its FFT reads are done), then two mel bands
        // per lane
        float* P = reinterpret_cast<float*>(S);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          P[lane + 64 * j] = r[2 * j];
          P[NC - lane - 64 * j] = r[2 * j + 1];
        }
        if (lane == 0) P[NC / 2] = r[16];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int m = lane + 64 * q;
          float acc = 0.f;
          if (m < mel.n_mels) {
            const int st = mel.start[m], n = mel.len[m], wo2 = mel.woff[m];
            // four interleaved partial sums: four weight loads and FMAs in flight per step instead
            // of one serial chain over the band (up to 48-64 bins for the top bands)
            float a1 = 0.f, a2 = 0.f, a3 = 0.f;
            const float* wq = mel.w + wo2;
            const float* pq = P + st;
            int i = 0;
            for (; i + 4 <= n; i += 4) {
              acc += wq[i] * pq[i];
              a1 += wq[i + 1] * pq[i + 1];
              a2 += wq[i + 2] * pq[i + 2];
              a3 += wq[i + 3] * pq[i + 3];
            }
            for (; i < n; ++i) acc += wq[i] * pq[i];
            acc = (acc + a1) + (a2 + a3);
          }
          res[q] = acc;
        }
      }
    }
    STAMP(2);
    LDS_BARRIER();  // every FFT is done: the scratch becomes staging + the next span
    STAMP(3);
    {
      const int un = u + W;
      if (un < U)
        load_span<FMW>(x + (long long)clip_of(un) * L, L, frame0_of(un) * hop - NFFT / 2, sp, pad_mode,
                  span, wave, lane);
    }
    STAMP(7);
    if constexpr (CPLX) {
      // frame-major rows are contiguous: each lane stores its 17 bins straight from registers
      // (a fixed count of buffer stores, dropped for a frame past the clip), no staging
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(out + (long long)b * T * NB * 2, (short)0,
                                                       clip_bytes, 0x00020000);
      const bool ok = fl < nfr;
      const int fo = (f0 + fl) * NB;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int oa = ok ? (fo + lane + 64 * j) * 8 : clip_bytes;
        const int ob = ok ? (fo + NC - lane - 64 * j) * 8 : clip_bytes;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, make_float2(xc[2 * j].x, xc[2 * j].y)), rs, oa, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, make_float2(xc[2 * j + 1].x, xc[2 * j + 1].y)), rs, ob, 0, 0);
      }
      const int om = (ok && lane == 0) ? (fo + NC / 2) * 8 : clip_bytes;
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, make_float2(xc[16].x, xc[16].y)), rs, om, 0, 0);
      continue;
    }
    if (fl < nfr) {
      if (!MELM) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          Sf[stage_pos<FPB>(fl, lane + 64 * j)] = res[2 * j];
          if (lane + j > 0) Sf[stage_pos<FPB>(fl, NC - lane - 64 * j)] = res[2 * j + 1];
        }
        if (lane == 0) Sf[stage_pos<FPB>(fl, NC / 2)] = res[16];
      } else {
        float* row = Sf + fl * RSTR_MEL;
        row[lane] = res[0];
        row[lane + 64] = res[1];
      }
    }
    STAMP(8);
    LDS_BARRIER();
    STAMP(4);
    const int nr = MELM ? mel.n_mels : NC;  // staged rows (bin 1024 goes straight out)
    float* oc = out + (long long)b * nrows * rowT;
    if (V4) {
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(oc, (short)0, clip_bytes, 0x00020000);
      constexpr int NQ = FPB / 4;  // 4-frame quads per row
      const int q = tid & (NQ - 1);
      // (row, quad) items: 1024 x NQ over 64 FMW threads = four per thread (MELM: 128 x NQ, one
      // for FMW = 16 and NQ * 128 / 512 = one for FMW = 8)
#pragma unroll
      for (int i = 0; i < (MELM ? 1 : 4); ++i) {
        const int k = tid / NQ + (64 * FMW / NQ) * i;
        float vv[4];
#pragma unroll
        for (int w = 0; w < 4; ++w)
          vv[w] = MELM ? Sf[(4 * q + w) * RSTR_MEL + k] : Sf[stage_pos<FPB>(4 * q + w, k)];
        const bool ok = k < nr && 4 * q + 3 < nfr;
        const int off = ok ? (int)((k * rowT + f0 + 4 * q) * 4) : clip_bytes;
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned,
                               make_float4(vv[0], vv[1], vv[2], vv[3])),
            rs, off, 0, 0);
      }
      if (!MELM) {  // bin 1024 of this wave's frame (lane 0 holds it)
        const int off = (lane == 0 && fl < nfr) ? (int)((NC * rowT + f0 + fl) * 4) : clip_bytes;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(res[1]), rs, off, 0, 0);
      }
    } else {
      float* ob = oc + f0;
      for (int e = tid; e < nr * (FPB / 4); e += blockDim.x) {
        const int k = e / (FPB / 4), q = e % (FPB / 4);
        for (int w = 0; w < 4 && 4 * q + w < nfr; ++w)
          ob[(long long)k * rowT + 4 * q + w] =
              MELM ? Sf[(4 * q + w) * RSTR_MEL + k] : Sf[stage_pos<FPB>(4 * q + w, k)];
      }
      if (!MELM && lane == 0 && fl < nfr) ob[NC * rowT + fl] = res[1];
    }
    STAMP(5);
    STAMP(6);
  }
}

// ---------------------------------------------------------------------------
// iSTFT (librosa.istft, center=True, Hann): workgroup = 512 threads, output segment of
// SEG = 16 samples per thread. Frames overlapping the segment are inverse-FFT'd 8 at a
// time (one per wave) into the waves' scratch; every thread then accumulates its own
// samples frame by frame in increasing frame order (deterministic OLA), together with
// the window-sum-square, and divides at the end.
//
// Spectrum input is frame-major complex (B, T, F, 2). With `prev` the spectrum used is
// normalise(cur - beta*prev) (Griffin-Lim momentum, librosa.griffinlim); with `mag`
// (B, T, F) it is multiplied by the magnitude; cur == NULL means all-ones phases.
// ---------------------------------------------------------------------------
constexpr int ISEG = 512 * 16;

__device__ __forceinline__ c2 gl_bin(const float2* cur, const float2* prev, const float* mag,
                                     long long base, int k, float beta, bool normalize) {
  c2 a = cur ? mk(cur[base + k].x, cur[base + k].y) : mk(1.f, 0.f);
  if (prev) {
    float2 pv = prev[base + k];
    a = a - mk(pv.x, pv.y) * beta;
  }
  if (normalize) {
    const float inv = __builtin_amdgcn_rcpf(sqrtf(a.x * a.x + a.y * a.y) + 1e-16f);
    a = mk(a.x * inv, a.y * inv);
  }
  if (mag) a = a * mag[base + k];
  return a;
}

// floor(x / d) for 0 <= x < 2^24 via a float reciprocal and one correction step.
__device__ __forceinline__ int div_hop(int x, int d, float inv) {
  int q = (int)((float)x * inv);
  const int r = x - q * d;
  if (r < 0) --q;
  else if (r >= d) ++q;
  return q;
}

// OLA per round: every thread owns 16 output samples sp = plo + tid + 512 i (padded
// coordinates); frame f covers sp when 0 <= sp - f*hop < NFFT. Each wave leaves its frame's
// windowed, 1/NC-scaled samples in its scratch, and every thread adds, for each of its samples,
// only the frames of this round that cover it (in increasing frame order). The
// window-sum-square of interior samples depends on sp mod hop only (table wssr, built once
// per workgroup in the same summation order); samples near the clip ends sum it directly.
__global__ __launch_bounds__(512, 2) void istft_kernel(const float2* __restrict__ cur,
                                                       const float2* __restrict__ prev,
                                                       const float* __restrict__ mag, float beta,
                                                       int normalize, int T, int hop,
                                                       float* __restrict__ y) {
  __shared__ __attribute__((aligned(16))) c2 scratch[WAVES * SCR];
  __shared__ c2 qt[QT];
  __shared__ c2 eht[64];
  __shared__ float wssr[512];
  const int b = blockIdx.y;
  const int L = hop * (T - 1);
  const int s0 = blockIdx.x * ISEG;  // segment start (unpadded coords)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  build_qtable(qt);
  if (threadIdx.x < 64) eht[threadIdx.x] = mk(kEh.e[threadIdx.x].x, kEh.e[threadIdx.x].y);
  __syncthreads();
  const int K = NFFT / hop;  // frames covering an interior sample (when hop divides NFFT)
  const bool table = (NFFT % hop) == 0 && hop <= 512;
  if (table) {
    for (int r = threadIdx.x; r < hop; r += blockDim.x) {
      float s = 0.f;
      for (int k = K - 1; k >= 0; --k) {  // frames in increasing order: m decreasing
        const float w = hann_w(qt, r + hop * k);
        s += w * w;
      }
      wssr[r] = s;
    }
  }
  c2* S = scratch + wave * SCR;
  const int plo = s0 + NFFT / 2, phi = s0 + NFFT / 2 + ISEG;  // padded range [plo, phi)
  int flo = (plo - NFFT) >= 0 ? (plo - NFFT) / hop + 1 : 0;
  int fhi = (phi - 1) / hop;  // frame f starts at f*hop < phi
  if (fhi > T - 1) fhi = T - 1;
  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  const bool norm = normalize != 0;
  const c2 e1 = tw<false>(qt, lane);  // W2048^lane
  const float scale = 1.f / NC;
  const float inv_hop = 1.f / (float)hop;
  for (int fb = flo; fb <= fhi; fb += WAVES) {
    const int f = fb + wave;
    if (f <= fhi) {
      const long long base = ((long long)b * T + f) * NB;
      // Stage the frame's 1025 updated bins in this wave's scratch: each bin is loaded and
      // phase-updated once (the packed signal below needs bins k and NC - k, which live in
      // different lanes), and no FFT registers are live yet, so all the loads are in flight
      // together.
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int k = lane + 64 * j;
        S[k] = gl_bin(cur, prev, mag, base, k, beta, norm);
      }
      if (lane == 0) S[NC] = gl_bin(cur, prev, mag, base, NC, beta, norm);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      c2 v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int k = lane + 64 * j;
        c2 Xk = S[k];
        c2 Xn = S[NC - k];
        if (k == 0) {
          Xk.y = 0.f;  // irfft ignores the imaginary part of DC and Nyquist
          Xn.y = 0.f;
        }
        c2 Xc = conj(Xn);
        c2 xe = (Xk + Xc) * 0.5f;
        c2 xo = cmul(Xk - Xc, conj(tw_bin(e1, j))) * 0.5f;
        v[j] = xe + mk(-xo.y, xo.x);  // Xe + i Xo
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();  // every lane has read the bins before the FFT reuses S
      fft1024<true>(v, S, qt, lane);
      // window (sin^2 form, as the STFT) and 1/NC, in place: S[n] = (x[2n], x[2n+1])
      const c2 eh = eht[lane];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int n = lane + 64 * j;
        const c2 z = S[n];
        S[n] = mk(z.x * (hann_sq(e1, j) * scale), z.y * (hann_sq(eh, j) * scale));
      }
    }
    __syncthreads();
    const int fe = min(fb + WAVES - 1, fhi);
    // An opaque zero keeps the per-sample values below from being hoisted out of the frame
    // loop (16 of them live across the FFT would not fit 128 VGPRs).
    int zero;
    asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int sp = plo + threadIdx.x + 512 * i + zero;
      const int q = div_hop(sp, hop, inv_hop);     // last frame covering sp
      const int f_first = max(fb, q - (NFFT - 1) / hop);
      const int f_last = min(fe, q);
      for (int fr = f_first; fr <= f_last; ++fr) {
        const int m = sp - fr * hop;
        if (m < NFFT) acc[i] += reinterpret_cast<const float*>(scratch + (fr - fb) * SCR)[m];
      }
    }
    __syncthreads();
  }
  float* yr = y + (long long)b * L;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int s = s0 + threadIdx.x + 512 * i;
    if (s >= L) continue;
    const int sp = s + NFFT / 2;
    const int q = sp / hop;
    const int fmin = (sp - NFFT) >= 0 ? (sp - NFFT) / hop + 1 : 0;  // first frame covering sp
    float wss;
    if (table && fmin == q - K + 1 && q <= T - 1) {
      wss = wssr[sp - q * hop];
    } else {
      wss = 0.f;
      for (int fr = fmin; fr <= min(q, T - 1); ++fr) {
        const float w = hann_w(qt, sp - fr * hop);
        wss += w * w;
      }
    }
    yr[s] = wss > 1.17549435e-38f ? acc[i] / wss : acc[i];
  }
}

// Griffin-Lim's iSTFT in two passes (the workspace holds the windowed frames):
//   ifft_frames_kernel: one wave per frame, 4 waves per workgroup, no workgroup barriers and
//     <= 128 VGPRs, so 4 waves/SIMD keep loads and FFTs of different frames overlapped; each
//     frame is inverse-FFT'd once (the fused istft_kernel recomputes 7 halo frames per
//     8192-sample segment and runs at 2 waves/SIMD). Writes the windowed, 1/NC-scaled frame.
//   ola_kernel: every output sample sums its covering frames in increasing order and divides
//     by the window-sum-square, the same arithmetic in the same order as istft_kernel, so the
//     two paths agree bitwise.
constexpr int IFW = 4;  // waves (frames in flight) per ifft_frames workgroup

// gl_bin for bin k = lane + 64 j of one frame through buffer descriptors: the per-lane byte
// offset is one VGPR and the j part a scalar soffset, so the frame's 48 loads can all be in
// flight without 48 64-bit addresses (which pushed the kernel past 128 VGPRs into scratch).
struct FrameBins {
  __amdgpu_buffer_rsrc_t c, p, m;
  bool has_c, has_p, has_m, norm;
  float beta;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t frame_rsrc(const void* ptr, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(ptr), (short)0, bytes, 0x00020000);
}

__device__ __forceinline__ c2 gl_bin_b(const FrameBins& fb, int lane, int k_sc) {
  c2 a = mk(1.f, 0.f);
  if (fb.has_c) {
    const auto u = __builtin_amdgcn_raw_buffer_load_b64(fb.c, lane * 8, k_sc * 8, 0);
    a = mk(__builtin_bit_cast(float, (unsigned)u[0]), __builtin_bit_cast(float, (unsigned)u[1]));
  }
  if (fb.has_p) {
    const auto u = __builtin_amdgcn_raw_buffer_load_b64(fb.p, lane * 8, k_sc * 8, 0);
    a = a - mk(__builtin_bit_cast(float, (unsigned)u[0]), __builtin_bit_cast(float, (unsigned)u[1])) * fb.beta;
  }
  if (fb.norm) {
    const float inv = __builtin_amdgcn_rcpf(sqrtf(a.x * a.x + a.y * a.y) + 1e-16f);
    a = mk(a.x * inv, a.y * inv);
  }
  if (fb.has_m)
    a = a * __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(fb.m, lane * 4, k_sc * 4, 0));
  return a;
}
constexpr int IFR = 1;  // frames per wave (more: the compiler hoists per-j constants out of the loop and spills)

__global__ __launch_bounds__(256, 4) void ifft_frames_kernel(const float2* __restrict__ cur,
                                                             const float2* __restrict__ prev,
                                                             const float* __restrict__ mag,
                                                             float beta, int normalize, int T,
                                                             float* __restrict__ frames) {
  __shared__ __attribute__((aligned(16))) c2 scratch[IFW * SCR];
  __shared__ c2 qt[QT];
  __shared__ c2 eht[64];
  const int b = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  build_qtable(qt);
  if (threadIdx.x < 64) eht[threadIdx.x] = mk(kEh.e[threadIdx.x].x, kEh.e[threadIdx.x].y);
  __syncthreads();
  c2* S = scratch + wave * SCR;
  const bool norm = normalize != 0;
  const c2 e1 = tw<false>(qt, lane);
  const c2 eh = eht[lane];
  const float scale = 1.f / NC;
#pragma unroll 1
  for (int r = 0; r < IFR; ++r) {
    const int f = (blockIdx.x * IFR + r) * IFW + wave;
    if (f >= T) break;  // wave-uniform; no workgroup barrier follows
    const long long base = ((long long)b * T + f) * NB;
    FrameBins fbn;
    fbn.has_c = cur != nullptr;
    fbn.has_p = prev != nullptr;
    fbn.has_m = mag != nullptr;
    fbn.norm = norm;
    fbn.beta = beta;
    fbn.c = frame_rsrc(cur ? cur + base : nullptr, NB * 8);
    fbn.p = frame_rsrc(prev ? prev + base : nullptr, NB * 8);
    fbn.m = frame_rsrc(mag ? mag + base : nullptr, NB * 4);
#pragma unroll
    for (int j = 0; j < 16; ++j) S[lane + 64 * j] = gl_bin_b(fbn, lane, 64 * j);
    if (lane == 0) S[NC] = gl_bin_b(fbn, 0, NC);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // opaque copies: the per-j twiddles and window values are formed where they are used,
    // not hoisted across the FFT (which would push the kernel past 128 VGPRs)
    c2 e1a = e1;
    asm volatile("" : "+v"(e1a.x), "+v"(e1a.y));
    c2 v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int k = lane + 64 * j;
      c2 Xk = S[k];
      c2 Xn = S[NC - k];
      if (k == 0) {
        Xk.y = 0.f;
        Xn.y = 0.f;
      }
      c2 Xc = conj(Xn);
      c2 xe = (Xk + Xc) * 0.5f;
      c2 xo = cmul(Xk - Xc, conj(tw_bin(e1a, j))) * 0.5f;
      v[j] = xe + mk(-xo.y, xo.x);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    fft1024<true>(v, S, qt, lane);
    float2* o = reinterpret_cast<float2*>(frames + ((long long)b * T + f) * NFFT);
    c2 e1b = e1, ehb = eh;
    asm volatile("" : "+v"(e1b.x), "+v"(e1b.y), "+v"(ehb.x), "+v"(ehb.y));
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int n = lane + 64 * j;
      const c2 z = S[n];
      o[n] = make_float2(z.x * (hann_sq(e1b, j) * scale), z.y * (hann_sq(ehb, j) * scale));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();  // S is restaged by the next frame
  }
}

constexpr int OLA_S = 4;  // samples per thread

__global__ __launch_bounds__(256) void ola_kernel(const float* __restrict__ frames, int T, int hop,
                                                  float* __restrict__ y) {
  __shared__ c2 qt[QT];
  __shared__ float wssr[512];
  const int b = blockIdx.y;
  const int L = hop * (T - 1);
  build_qtable(qt);
  __syncthreads();
  const int K = NFFT / hop;
  const bool table = (NFFT % hop) == 0 && hop <= 512;
  if (table) {
    for (int r = threadIdx.x; r < hop; r += blockDim.x) {
      float s = 0.f;
      for (int k = K - 1; k >= 0; --k) {  // frames in increasing order, as istft_kernel
        const float w = hann_w(qt, r + hop * k);
        s += w * w;
      }
      wssr[r] = s;
    }
  }
  __syncthreads();
  const float* fb = frames + (long long)b * T * NFFT;
  float* yr = y + (long long)b * L;
#pragma unroll
  for (int i = 0; i < OLA_S; ++i) {
    const int s = (blockIdx.x * OLA_S + i) * 256 + threadIdx.x;
    if (s >= L) break;
    const int sp = s + NFFT / 2;
    const int q = sp / hop;
    const int fmin = (sp - NFFT) >= 0 ? (sp - NFFT) / hop + 1 : 0;
    const int fmax = min(q, T - 1);
    float acc = 0.f;
    for (int fr = fmin; fr <= fmax; ++fr) acc += fb[(long long)fr * NFFT + (sp - fr * hop)];
    float wss;
    if (table && fmin == q - K + 1 && q <= T - 1) {
      wss = wssr[sp - q * hop];
    } else {
      wss = 0.f;
      for (int fr = fmin; fr <= fmax; ++fr) {
        const float w = hann_w(qt, sp - fr * hop);
        wss += w * w;
      }
    }
    yr[s] = wss > 1.17549435e-38f ? acc / wss : acc;
  }
}

// ---------------------------------------------------------------------------
// Griffin-Lim synthesis in one pass (round 2): spectra -> signal without the frames workspace.
// The two-pass iSTFT above moves every windowed frame through HBM twice (written by
// ifft_frames_kernel, read back by ola_kernel: 1 GB per iteration at config 2, on top of the
// 1.3 GB of spectra), and the fused istft_kernel recomputes 7 halo frames per 32. Here a
// workgroup (8 waves) owns G consecutive frames of one clip and every sample they cover
// (<= 8192, 16 per thread, in registers):
//   per round of 8 frames, wave w: bins of frame f = X = mag * normalise(cur - beta prev)
//     (issued one round ahead, during the previous round's overlap-add), staged in the wave's
//     LDS scratch for the irfft pre-twist (bins k and 1024 - k live in different lanes), the
//     inverse 1024-point FFT as conj(fft1024_v2p(conj v))
//     (twiddles from two table values: the LDS holds the 8 frames), window and 1/1024 into the
//     wave's LDS scratch; barrier; every thread adds the round's frames covering its samples
//     in increasing frame order.
//   end: samples whose covering frames all belong to the workgroup are final (divided by the
//     window-sum-square); the NFFT - hop samples shared with a neighbour (a "seam") go out as
//     partial sums, and gl_seam_kernel adds the two halves (earlier frames first) and divides.
//     (Finishing a seam in whichever workgroup arrives second needs a device-scope release /
//     acquire: on gfx950 that writes back the XCD's L2, and the kernel ran 8x slower.)
// Reads each bin once (20 B: cur, prev, mag), writes each sample once.
// ---------------------------------------------------------------------------
constexpr int GLW = 8;                      // waves per synthesis workgroup
constexpr int GL_OWN = 12;                  // samples per thread (G = 16 frames at hop 256)
constexpr int GL_SEG = 64 * GLW * GL_OWN;   // samples a workgroup covers (8192)

// frames per workgroup: the covered span (G - 1) hop + NFFT fits GL_SEG; whole rounds when G >= 8
static inline int gl_frames(int hop) {
  const int g = (GL_SEG - NFFT) / hop + 1;
  static const int cap = [] {  // MST_GL_FRAMES: a smaller G (A/B tuning)
    const char* e = getenv("MST_GL_FRAMES");
    return e ? atoi(e) : 0;
  }();
  int gg = cap > 0 && cap < g ? cap : g;
  gg = gg >= GLW ? gg / GLW * GLW : gg;
  // G hop >= NFFT - hop: no sample is covered by more than two workgroups, so a seam is the sum
  // of exactly two atomic adds (order-independent)
  return max(gg, ceil_div(NFFT - hop, hop));
}

// Squared periodic Hann, sin^4(pi n / 2048) (the sin^2 form of the synthesis window), into an
// LDS table: computed, not looked up, so no load latency sits at the start of a workgroup.
__device__ __forceinline__ void gl_fill_h2(float* h2) {
  for (int n = threadIdx.x; n < NFFT; n += blockDim.x) {
    const float sn = sinpif((float)n * (1.f / NFFT));
    h2[n] = (sn * sn) * (sn * sn);
  }
}

// window-sum-square at padded sample sp, frames in increasing order
__device__ __forceinline__ float gl_wss(const float* h2, int sp, int fmin, int fmax, int hop) {
  float s = 0.f;
  for (int fr = fmin; fr <= fmax; ++fr) s += h2[sp - fr * hop];
  return s;
}

// One frame's raw bins in registers (issued a round ahead, consumed by gl_frame_x).
struct GlRaw {
  float2 c[17], p[17];
};

__device__ __forceinline__ float2 gl_ld2(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}

// Issue frame f's bin loads (k = lane + 64 j, and bin 1024 in every lane as entry 16). Always
// issued (a frame past the workgroup's range reads zeros through an empty descriptor): a
// conditional refill would keep the previous values live across the FFT.
__device__ __forceinline__ void gl_issue(const float2* cur, const float2* prev, int b, int T,
                                         int f, bool valid, int lane, GlRaw& r) {
  const long long base = ((long long)b * T + (valid ? f : 0)) * NB;
  // absent operands (cur == NULL: all-ones phases; prev == NULL: no momentum) read zeros too
  const auto rc = frame_rsrc(cur ? cur + base : nullptr, valid && cur ? NB * 8 : 0);
  const auto rp = frame_rsrc(prev ? prev + base : nullptr, valid && prev ? NB * 8 : 0);
#pragma unroll
  for (int j = 0; j < 16; ++j) r.c[j] = gl_ld2(rc, lane * 8, 64 * j * 8);
  r.c[16] = gl_ld2(rc, 0, NC * 8);
#pragma unroll
  for (int j = 0; j < 16; ++j) r.p[j] = gl_ld2(rp, lane * 8, 64 * j * 8);
  r.p[16] = gl_ld2(rp, 0, NC * 8);
}

// frame f's magnitudes (loaded when the frame is synthesised, not a round ahead: registers)
__device__ __forceinline__ float gl_mag(__amdgpu_buffer_rsrc_t rm, int lane, int j) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rm, j < 16 ? lane * 4 : 0,
                                                                        j < 16 ? 64 * j * 4 : NC * 4, 0));
}

// X = mag * normalise(cur - beta prev) (gl_bin's arithmetic) for entry j
__device__ __forceinline__ c2 gl_x(const GlRaw& r, float mg, int j, bool has_c, bool has_p,
                                   bool norm, float beta) {
  c2 a = has_c ? mk(r.c[j].x, r.c[j].y) : mk(1.f, 0.f);
  if (has_p) a = a - mk(r.p[j].x, r.p[j].y) * beta;
  if (norm) {
    const float inv = __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(a.x * a.x + a.y * a.y) + 1e-16f);
    a = mk(a.x * inv, a.y * inv);
  }
  return a * mg;
}

// LDS-only workgroup barrier: __syncthreads() would also drain vmcnt, i.e. wait for the next
// round's bin loads issued just before the overlap-add
#define GL_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")

__global__ __launch_bounds__(512, 4) void gl_synth_kernel(const float2* __restrict__ cur,
                                                          const float2* __restrict__ prev,
                                                          const float* __restrict__ mag,
                                                          float beta, int normalize, int T,
                                                          int hop, int G, int nwg,
                                                          float* __restrict__ y,
                                                          float* __restrict__ ynext) {
  __shared__ __attribute__((aligned(16))) c2 scratch[GLW * SCR];
  __shared__ float h2[NFFT];
  const int b = blockIdx.y, wg = blockIdx.x;
  const int F0 = wg * G, F1 = min(T, F0 + G);
  const int L = hop * (T - 1);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  gl_fill_h2(h2);  // read after the loop's barriers
  c2* S = scratch + wave * SCR;
  const float* Sf = reinterpret_cast<const float*>(scratch);
  const int c0 = F0 * hop;  // padded coordinate of the first covered sample
  float acc[GL_OWN];
#pragma unroll
  for (int i = 0; i < GL_OWN; ++i) acc[i] = 0.f;
  const float inv_hop = 1.f / (float)hop;
  const bool has_c = cur != nullptr, has_p = prev != nullptr, norm = normalize != 0;
  const c2 eh = mk(kEh.e[threadIdx.x & 63].x, kEh.e[threadIdx.x & 63].y);  // W4096^(2 lane + 1)
  GlRaw rb;
  gl_issue(cur, prev, b, T, F0 + wave, F0 + wave < F1, threadIdx.x & 63, rb);
#pragma unroll 1
  for (int fb = F0; fb < F1; fb += GLW) {
    const int f = fb + wave;
    if (f < F1) {
      int tid = threadIdx.x;
      __asm__ volatile("" : "+v"(tid));  // lane values formed here, not hoisted out of the loop
      const int lane = tid & 63;
      const float2 e1f = kFftTabs.p[lane], wbf = kFftTabs.p[32 * (lane & 15)];  // W2048^lane, W64^(lane & 15)
      const auto rm = frame_rsrc(mag + ((long long)b * T + f) * NB, NB * 4);
      float mg[17];
#pragma unroll
      for (int j = 0; j < 17; ++j) mg[j] = gl_mag(rm, lane, j);
      // X staged in the wave's scratch (each bin formed once; the pre-twist pairs k with
      // 1024 - k, which live in different lanes)
#pragma unroll
      for (int j = 0; j < 16; ++j) S[lane + 64 * j] = gl_x(rb, mg[j], j, has_c, has_p, norm, beta);
      if (lane == 0) S[NC] = gl_x(rb, mg[16], 16, has_c, has_p, norm, beta);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const c2 e1 = mk(e1f.x, e1f.y);
      // irfft pre-twist: v[k] = Xe + i Xo, Xe = (X_k + conj X_{1024-k}) / 2,
      // Xo = (X_k - conj X_{1024-k}) conj(W2048^k) / 2
      c2 V[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int k = lane + 64 * j;
        c2 Xk = S[k];
        c2 Xn = S[NC - k];
        if (k == 0) {  // irfft ignores the imaginary parts of DC and Nyquist
          Xk.y = 0.f;
          Xn.y = 0.f;
        }
        const c2 Xc = conj(Xn);
        const c2 xe = (Xk + Xc) * 0.5f;
        const c2 xo = cmul(Xk - Xc, conj(tw_bin(e1, j))) * 0.5f;
        const c2 v = xe + mk(-xo.y, xo.x);
        V[j] = conj(v);  // inverse FFT = conj(FFT(conj v))
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();  // every lane has read the bins before the FFT reuses S
      fft1024_v2p(V, S, cmul(e1, e1), mk(wbf.x, wbf.y), lane);
      const float scale = 1.f / NC;
#pragma unroll
      for (int j = 0; j < 16; ++j) {  // z[n] = conj(V[j]), n = lane + 64 j: samples 2n, 2n + 1
        const c2 u = V[j];
        S[lane + 64 * j] = mk(u.x * (hann_sq(e1, j) * scale), -u.y * (hann_sq(eh, j) * scale));
      }
    }
    GL_BARRIER();
    // the next round's bins are in flight during the overlap-add below
    gl_issue(cur, prev, b, T, fb + GLW + wave, fb + GLW + wave < F1, threadIdx.x & 63, rb);
    const int fe = min(fb + GLW, F1) - 1;
    int zero;
    asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
    // frame-stationary: for each of the round's frames (in increasing order) and each block of
    // the wave's 64 samples, a wave-uniform test on the block's offset m0 in the frame: fully
    // inside adds without a per-lane check, partly inside with one, outside skips
    const int wbase = c0 + 64 * wave;
    const int lane4 = (threadIdx.x & 63) + zero;
    for (int fr = fb; fr <= fe; ++fr) {
      const float* Fr = Sf + (fr - fb) * (2 * SCR) + lane4;
      const int m00 = wbase - fr * hop;
#pragma unroll
      for (int i = 0; i < GL_OWN; ++i) {
        const int m0 = m00 + 512 * i;  // wave-uniform
        if (m0 + 63 < 0 || m0 >= NFFT) continue;
        if (m0 >= 0 && m0 + 63 < NFFT) {
          acc[i] += Fr[m0];
        } else {
          const int m = m0 + lane4;
          if ((unsigned)m < (unsigned)NFFT) acc[i] += Fr[m0];
        }
      }
    }
    GL_BARRIER();
  }
  const int cov_end = (F1 - 1) * hop + NFFT;
  float* yr = y + (long long)b * L;
  float* yn = ynext ? ynext + (long long)b * L : nullptr;
#pragma unroll
  for (int i = 0; i < GL_OWN; ++i) {
    const int sp = c0 + threadIdx.x + 512 * i;
    if (sp >= cov_end) continue;
    const int s = sp - NFFT / 2;
    if (s < 0 || s >= L) continue;
    const int fmin = (sp - NFFT) >= 0 ? div_hop(sp - NFFT, hop, inv_hop) + 1 : 0;
    const int fmax = min(div_hop(sp, hop, inv_hop), T - 1);
    const float wss = gl_wss(h2, sp, fmin, fmax, hop);
    const float v = wss > 1.17549435e-38f ? acc[i] * __builtin_amdgcn_rcpf(wss) : acc[i];
    const bool right = F1 < T && fmax >= F1;  // shared with the next workgroup
    if ((F0 > 0 && fmin < F0) || right) {
      // a seam sample: exactly two workgroups add into a zeroed word, and a + b = b + a in
      // IEEE arithmetic, so the result does not depend on which arrives first
      unsafeAtomicAdd(yr + s, v);
      if (right && yn) yn[s] = 0.f;  // the next synthesis target's seam starts from zero
    } else {
      yr[s] = v;
    }
  }
}

// (B, F, T) -> (B, T, F) with optional log-power -> magnitude (inference.py:109).
__global__ void transpose_mag_kernel(const float* __restrict__ S, int F, int T, int mag_from_logpow,
                                     float* __restrict__ St) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z;
  const int f0 = blockIdx.y * 32, t0 = blockIdx.x * 32;
  const float* Sb = S + (long long)b * F * T;
  for (int i = threadIdx.y; i < 32; i += blockDim.y) {
    int f = f0 + i, t = t0 + threadIdx.x;
    float v = (f < F && t < T) ? Sb[(long long)f * T + t] : 0.f;
    if (mag_from_logpow) v = sqrtf(expm1f(fminf(fmaxf(v, 0.f), 20.f)));
    tile[i][threadIdx.x] = v;
  }
  __syncthreads();
  float* Ob = St + (long long)b * F * T;
  for (int i = threadIdx.y; i < 32; i += blockDim.y) {
    int t = t0 + i, f = f0 + threadIdx.x;
    if (f < F && t < T) Ob[(long long)t * F + f] = tile[threadIdx.x][i];
  }
}

int stft_launch(int mode, const float* x, int B, int L, int n_fft, int hop, int pad_mode, float* out,
                MelTab mel, hipStream_t st) {
  MST_REQUIRE(x && out && B > 0 && n_fft == NFFT && hop > 0);
  MST_REQUIRE(L > NFFT / 2 || pad_mode == MST_PAD_CONSTANT);
  MST_REQUIRE(pad_mode == MST_PAD_REFLECT || pad_mode == MST_PAD_CONSTANT);
  const int T = 1 + L / hop;
  // frames per block: 16 (one 1024-thread workgroup per CU, 64-byte row pieces) for the
  // log-power / power STFT, 8 (two workgroups per CU) for mel and the complex STFT
  // (profiles/r03/ab_fm16.txt: log-power 0.166 -> 0.162 ms; mel +2 %, Griffin-Lim +8 % at 16)
  const int fmw = (mode == MODE_LOGPOW || mode == MODE_POWER) ? FM_WAVES_POW : FM_WAVES;
  const bool fm_fits = !(hop & 1) && (long long)((fmw - 1) * hop + NFFT) * 4 <= (long long)fmw * (SCR * 8 - NC * 4);
  if (mode == MODE_COMPLEX && !fm_fits) {  // frame-major (B, T, F, 2), round-1 kernel
    dim3 grid(ceil_div(T, FR), B), block(512);
    hipLaunchKernelGGL(stft_kernel<MODE_COMPLEX>, grid, block, 0, st, x, L, T, hop, pad_mode, out, mel);
  } else if (!fm_fits) {
    // odd hops (8-byte span reads) or spans beyond the scratch: the round-1 kernel
    dim3 grid(ceil_div(T, FR), B), block(512);
    switch (mode) {
      case MODE_LOGPOW: hipLaunchKernelGGL(stft_kernel<MODE_LOGPOW>, grid, block, 0, st, x, L, T, hop, pad_mode, out, mel); break;
      case MODE_POWER: hipLaunchKernelGGL(stft_kernel<MODE_POWER>, grid, block, 0, st, x, L, T, hop, pad_mode, out, mel); break;
      default: hipLaunchKernelGGL(stft_kernel<MODE_MEL>, grid, block, 0, st, x, L, T, hop, pad_mode, out, mel); break;
    }
  } else {  // frequency-major: persistent XCD-grouped workgroups over FM_WAVES-frame blocks
    // resident workgroups: 256 CUs x (1024 threads: one, 512: two), i.e. 32 or 64 per XCD group
    const long long per_group = (long long)ceil_div(B, 8) * ceil_div(T, fmw);
    const int wmax = fmw == 16 ? 32 : 64;
    const int W = (int)(per_group < wmax ? per_group : wmax);
    dim3 grid(8 * W), block(64 * fmw);
    const long long rows = mode == MODE_MEL ? mel.n_mels : NB;
    MST_REQUIRE(rows * T * (mode == MODE_COMPLEX ? 8 : 4) < (1ll << 31));  // per-clip buffer descriptors
    const bool v4 = mode == MODE_COMPLEX || ((T & 3) == 0 && ((uintptr_t)out & 15) == 0);
#define MST_STFT_FM(M, V) hipLaunchKernelGGL((stft_fm_kernel<M, V, FM_WAVES>), grid, block, 0, st, x, B, L, T, hop, pad_mode, out, mel, W)
#define MST_STFT_FMP(M, V) hipLaunchKernelGGL((stft_fm_kernel<M, V, FM_WAVES_POW>), grid, block, 0, st, x, B, L, T, hop, pad_mode, out, mel, W)
    switch (mode) {
      case MODE_LOGPOW: if (v4) MST_STFT_FMP(MODE_LOGPOW, true); else MST_STFT_FMP(MODE_LOGPOW, false); break;
      case MODE_POWER: if (v4) MST_STFT_FMP(MODE_POWER, true); else MST_STFT_FMP(MODE_POWER, false); break;
      case MODE_COMPLEX: MST_STFT_FM(MODE_COMPLEX, true); break;
      default: if (v4) MST_STFT_FM(MODE_MEL, true); else MST_STFT_FM(MODE_MEL, false); break;
    }
#undef MST_STFT_FM
#undef MST_STFT_FMP
  }
  MST_CHECK_LAUNCH();
  return MST_OK;
}

int istft_launch(const float2* cur, const float2* prev, const float* mag, float beta, int normalize,
                 int B, int T, int hop, float* y, hipStream_t st) {
  const int L = hop * (T - 1);
  dim3 grid(ceil_div(L, ISEG), B), block(512);
  hipLaunchKernelGGL(istft_kernel, grid, block, 0, st, cur, prev, mag, beta, normalize, T, hop, y);
  MST_CHECK_LAUNCH();
  return MST_OK;
}

// Two-pass iSTFT through a (B, T, NFFT) frames workspace (Griffin-Lim).
int istft2_launch(const float2* cur, const float2* prev, const float* mag, float beta,
                  int normalize, int B, int T, int hop, float* frames, float* y, hipStream_t st) {
  const int L = hop * (T - 1);
  hipLaunchKernelGGL(ifft_frames_kernel, dim3(ceil_div(T, IFW * IFR), B), dim3(64 * IFW), 0, st,
                     cur, prev, mag, beta, normalize, T, frames);
  MST_CHECK_LAUNCH();
  hipLaunchKernelGGL(ola_kernel, dim3(ceil_div(L, 256 * OLA_S), B), dim3(256), 0, st, frames, T,
                     hop, y);
  MST_CHECK_LAUNCH();
  return MST_OK;
}

// One-pass Griffin-Lim synthesis (gl_synth_kernel). Seam samples (shared by two workgroups) are
// added atomically into y, whose seams must be zero on entry; the launch zeroes the seams of
// `ynext` (the next synthesis target) as it goes.
static bool gl_one_pass(int hop) {  // hop > 1024: the two-pass frames-workspace path
  return hop <= 1024;
}

int gl_synth_launch(const float2* cur, const float2* prev, const float* mag, float beta,
                    int normalize, int B, int T, int hop, float* y, float* ynext, hipStream_t st) {
  const int G = gl_frames(hop);
  const int nwg = ceil_div(T, G);
  hipLaunchKernelGGL(gl_synth_kernel, dim3(nwg, B), dim3(64 * GLW), 0, st, cur, prev, mag, beta,
                     normalize, T, hop, G, nwg, y, ynext);
  MST_CHECK_LAUNCH();
  return MST_OK;
}


// ---------------------------------------------------------------------------
// Multi-scale spectral loss, n = 2048 (mss.hip has the other sizes and the plan): the same
// ownership, frame pairing and ordered overlap-add as mss_wave_body (mss.hip), with every transform a
// register-resident fft1024_v2.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int mss_reflect(int i, int L) {
  i = i < 0 ? -i : i;
  return i >= L ? 2 * (L - 1) - i : i;
}

// n = 2048: each frame of pred and of target is a real 2048-point transform, computed as the
// STFT does it: fft1024_v2 of z[n] = w[2n] x[2n] + i w[2n+1] x[2n+1] (n = lane + 64 j), then the
// real-FFT post-twist pairing bins k = l + 64 j and 1024 - k (partner Z in lane 64 - l, register
// 15 - j, by ds_bpermute). Pred and target are never packed into one complex signal: that leaves
// the target's spectrum with rounding noise of the pred's size, and a silent target then moves
// log(S + eps) (tools/mss_probe.py). The gradient frame g = Re sum_f Y_f e^(2 pi i f m / 2048)
// (Y Hermitian, Y_f = G_f / 2 for 0 < f < 1024, real Y_0, Y_1024) is one 1024-point inverse:
// z[n] = g[2n] + i g[2n+1] = IDFT1024(Z'), Z'_k = A + i e^(i pi k / 1024) B with
// A = Y_k + conj Y_(1024-k), B = Y_k - conj Y_(1024-k); Z'_(1024-k) = conj A + i conj(e B) goes to
// lane 64 - l, register 15 - j (lane 0 keeps its own). Frames a and b of a pair then sit in the
// wave's LDS buffer as (g_a, g_b) for the workgroup's ordered overlap-add. Two fft1024_v2 per
// frame (the target's magnitudes come from mss_target2048_kernel).
__device__ __forceinline__ c2 mss_term(c2 P, float st, bool use, bool grad, const MssArgs& a,
                                       float& s_abs, float& s_log) {
  const float sp = __builtin_amdgcn_sqrtf(P.x * P.x + P.y * P.y);
  c2 g2 = mk(0.f, 0.f);
  if (use) {
    s_abs += fabsf(sp - st);
    s_log += fabsf(__log2f(sp + a.eps) * 0.69314718055994531f - __log2f(st + a.eps) * 0.69314718055994531f);
    if (grad && sp > 0.f) {
      const float sg = sp > st ? 1.f : (sp < st ? -1.f : 0.f);
      const float g = sg * (1.f + a.alpha * __builtin_amdgcn_rcpf(sp + a.eps)) * a.inv_cnt;
      g2 = P * (g * __builtin_amdgcn_rcpf(sp));
    }
  }
  return g2;
}

// 2 X[k] and 2 conj X[1024 - k] for k = l + 64 j (j < 8) from Z in v (power_pairs_v2's pairing)
__device__ __forceinline__ void real_pairs(const c2 v[16], const FftTabs& tb, int lane, int src,
                                           c2 xk[8], c2 xm[8]) {
  c2 prev = v[0];  // lane 0's partner 1024 - 64 j is its own v[16 - j] (v[0] for j = 0)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const c2 bpj = mk(bperm(src, v[15 - j].x), bperm(src, v[15 - j].y));
    const c2 Bq = lane == 0 ? prev : bpj;
    prev = bpj;
    const c2 A = v[j];
    const c2 E = mk(A.x + Bq.x, A.y - Bq.y);
    const c2 D = mk(A.y + Bq.y, Bq.x - A.x);  // -i (A - conj(Bq))
    const float2 w = tb.p[lane + 64 * j];
    const c2 TD = cmul(mk(w.x, w.y), D);
    xk[j] = (E + TD) * 0.5f;     // X[k]
    xm[j] = conj(E - TD) * 0.5f;  // X[1024 - k]
  }
}

__global__ __launch_bounds__(256, 2) void mss_fft2048_kernel(const MssArgs a) {
  constexpr int N = 2048, H = N / 4, HALF = N / 2, W = 4, OWN = MSS_RWIN / 256;
  constexpr int SPILL = 3 * H / 256;  // per thread: samples past the range its frames reach
  __shared__ __attribute__((aligned(16))) c2 buf[W * N];  // per wave: FFT scratch, then G
  __shared__ __attribute__((aligned(16))) FftTabs tb;
  __shared__ float red[2][W];
  const int w = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int L = (int)a.L;
  const float* p = a.pred + (long long)b * a.L;
  const float* tm = a.tmag + (long long)b * a.T * (HALF + 1);  // float64-accurate |X_target|
  const bool grad = a.dpred != nullptr;
  {
    const float4* src = reinterpret_cast<const float4*>(&kFftTabs);
    float4* dst = reinterpret_cast<float4*>(&tb);
    for (int i = tid; i < TAB_F4; i += 256) dst[i] = src[i];
  }
  __syncthreads();
  auto hann = [&](int n) {  // periodic Hann 0.5 - 0.5 cos(2 pi n / 2048) = 0.5 - 0.5 Re W2048^n
    const float2 e = tb.p[n & 511];
    const int qd = (n >> 9) & 3;  // W^(512 qd + r) = (-i)^qd W^r
    const float re = qd == 0 ? e.x : (qd == 1 ? e.y : (qd == 2 ? -e.x : -e.y));
    return 0.5f - 0.5f * re;
  };
  const int own_lo = w * MSS_RWIN;
  const int f_own0 = w * (MSS_RWIN / H), f_own1 = min(f_own0 + MSS_RWIN / H, a.T);
  // frames [f_own0, f_own1) only (one round): the gradient of the last three on the 3H samples
  // past the range goes to a.spill (added by mss_sum_kernel / mss_fold, mss.hip), as in mss_wave_body
  const int f_lo = f_own0;
  c2* S = buf + wave * N;
  float acc[OWN + SPILL];  // sample own_lo + tid + 256 i (i >= OWN: past the range)
#pragma unroll
  for (int i = 0; i < OWN + SPILL; ++i) acc[i] = 0.f;
  float s_abs = 0.f, s_log = 0.f;

#pragma unroll 1
  for (int t_round = f_lo; t_round < f_own1; t_round += 2 * W) {
    const int t_base = t_round + 2 * wave;
    if (t_base < f_own1) {  // wave-uniform
      int tid2 = tid;
      __asm__ volatile("" : "+v"(tid2));
      const int lane = tid2 & 63;
      const int src = ((64 - lane) & 63) * 4;  // bperm partner: lane 64 - l
      c2 za[16];                               // frame a's gradient samples (g[2n], g[2n + 1])
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
        const int t = t_base + pass;
        const bool valid = t < f_own1;
        // the target's magnitudes at bins k = l + 64 j, 1024 - k and 512, loaded ahead of the FFT
        // (clamped frame: a past-the-end frame reads a valid row and is masked by `valid`)
        const float* tr = tm + (long long)min(t, a.T - 1) * (HALF + 1);
        float qk[8], qm[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          qk[j] = tr[lane + 64 * j];
          qm[j] = tr[HALF - lane - 64 * j];
        }
        const float q512 = tr[512];
        c2 vp[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int n = lane + 64 * j;
          vp[j] = mk(0.f, 0.f);
          if (valid) {
            const int s0 = t * H + 2 * n - HALF;
            const int i0 = mss_reflect(s0, L), i1 = mss_reflect(s0 + 1, L);
            const float h0 = hann(2 * n), h1 = hann(2 * n + 1);
            vp[j] = mk(h0 * p[i0], h1 * p[i1]);
          }
        }
        fft1024_v2(vp, S, tb, lane);  // Z_pred[l + 64 j]
        c2 pk[8], pm[8], yk[8], ym[8];
        real_pairs(vp, tb, lane, src, pk, pm);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          yk[j] = mss_term(pk[j], qk[j], valid, grad, a, s_abs, s_log) * 0.5f;
          // lane 0's X[1024 - 0] is the Nyquist bin X[1024] (xm[0]), its magnitude tr[1024]
          ym[j] = mss_term(pm[j], qm[j], valid, grad, a, s_abs, s_log) * 0.5f;
        }
        // f = 512: X[512] = conj Z[512] (lane 0, register 8)
        const c2 y512 = mss_term(conj(vp[8]), q512, valid && lane == 0, grad, a, s_abs, s_log) * 0.5f;
        if (!grad) continue;
        if (lane == 0) {  // Y_0, Y_1024 are real (and G_f / 2 -> G_f there)
          yk[0] = mk(2.f * yk[0].x, 0.f);
          ym[0] = mk(2.f * ym[0].x, 0.f);
        }
        c2 v[16], cn[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const c2 A = yk[j] + conj(ym[j]), B = yk[j] - conj(ym[j]);
          const float2 wk = tb.p[lane + 64 * j];
          const c2 C = cmul(mk(wk.x, -wk.y), B);  // e^(i pi k / 1024) B
          v[j] = mk(A.x - C.y, A.y + C.x);         // A + i C
          cn[j] = mk(A.x + C.y, -A.y + C.x);       // conj A + i conj C
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[15 - j] = mk(bperm(src, cn[j].x), bperm(src, cn[j].y));
        if (lane == 0) {  // lane 0 holds Z'_(64 r): Z'_512 = 2 conj Y_512, Z'_(1024 - 64 j) from itself
          v[8] = mk(2.f * y512.x, -2.f * y512.y);
#pragma unroll
          for (int j = 1; j < 8; ++j) v[16 - j] = cn[j];
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = conj(v[j]);
        fft1024_v2(v, S, tb, lane);  // conj(z) at n = l + 64 j
        if (pass == 0) {
#pragma unroll
          for (int j = 0; j < 16; ++j) za[j] = conj(v[j]);
        } else {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();  // the FFT's transpose reads of S are done
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const int n = lane + 64 * j;
            S[2 * n] = mk(za[j].x, v[j].x);       // g_a[2n], g_b[2n]
            S[2 * n + 1] = mk(za[j].y, -v[j].y);  // g_a[2n + 1], g_b[2n + 1]
          }
        }
      }
    }
    if (!grad) continue;
    __syncthreads();
    // frames th - q (q = 3 .. 0) at offset sp mod H + q H, four fixed steps (mss_wave_body)
    const int r_hi = min(t_round + 2 * W, f_own1);
    const int s_lo = t_round * H - own_lo, s_hi = (r_hi - 1) * H + N - own_lo;
#pragma unroll
    for (int i = 0; i < OWN + SPILL; ++i) {
      if (256 * (i + 1) <= s_lo || 256 * i >= s_hi) continue;
      const unsigned sp = own_lo + tid + 256 * i;
      const int th = (int)(sp / H);
      const unsigned jr = sp % H;
      float vv = acc[i];
#pragma unroll
      for (int q = 3; q >= 0; --q) {
        const int rel = th - q - t_round;
        const bool ok = rel >= 0 && rel < r_hi - t_round;
        const unsigned rc = ok ? rel : 0u, j = jr + q * H;
        const c2 g = buf[(rc >> 1) * N + j];
        vv = __builtin_fmaf(hann(j), ok ? ((rc & 1) ? g.y : g.x) : 0.f, vv);
      }
      acc[i] = vv;
    }
    __syncthreads();
  }

  s_abs = wave_sum(s_abs);
  s_log = wave_sum(s_log);
  if ((tid & 63) == 0) {
    red[0][wave] = s_abs;
    red[1][wave] = s_log;
  }
  __syncthreads();
  if (tid == 0) {
    float sa = 0.f, sl = 0.f;
    for (int i = 0; i < W; ++i) {
      sa += red[0][i];
      sl += red[1][i];
    }
    a.partial[((long long)b * a.nwg + w) * 2] = sa;
    a.partial[((long long)b * a.nwg + w) * 2 + 1] = sl;
  }
  if (!grad) return;
  float* dp = a.dpred + (long long)b * a.L;
  float* ed = a.edges + (long long)b * N;
  const int own_hi = min(own_lo + MSS_RWIN, L + N);
  // this size's gradient slab (the sizes are summed in order by mss_sum_kernel, mss.hip)
#pragma unroll
  for (int i = 0; i < OWN; ++i) {
    // one store per sample to the address picked by selects (stores under the three-way
    // branch each waited for every earlier store: vmcnt counts stores on gfx950)
    const int pp = own_lo + tid + 256 * i;
    const int x = pp - HALF;
    float* dst = x < 0 ? ed + pp : (x >= L ? ed + HALF + (x - L) : dp + x);
    if (pp < own_hi) *dst = acc[i];
  }
  float* spl = a.spill + ((long long)b * a.nwg + w) * (3 * H);
#pragma unroll
  for (int i = 0; i < SPILL; ++i) spl[tid + 256 * i] = acc[OWN + i];
}

}  // namespace

void mss_fft2048_launch(const MssArgs& a, unsigned nwg, unsigned B, hipStream_t st) {
  hipLaunchKernelGGL(mss_fft2048_kernel, dim3(nwg, B), dim3(256), 0, st, a);
}

extern "C" {

int mst_stft_logpow_f32(const float* x, int32_t B, int32_t L, int32_t n_fft, int32_t hop,
                        int32_t pad_mode, float* out, void* stream) {
  return stft_launch(MODE_LOGPOW, x, B, L, n_fft, hop, pad_mode, out, MelTab{}, (hipStream_t)stream);
}

int mst_stft_power_f32(const float* x, int32_t B, int32_t L, int32_t n_fft, int32_t hop,
                       int32_t pad_mode, float* out, void* stream) {
  return stft_launch(MODE_POWER, x, B, L, n_fft, hop, pad_mode, out, MelTab{}, (hipStream_t)stream);
}

int mst_stft_complex_f32(const float* x, int32_t B, int32_t L, int32_t n_fft, int32_t hop,
                         int32_t pad_mode, float* out, void* stream) {
  return stft_launch(MODE_COMPLEX, x, B, L, n_fft, hop, pad_mode, out, MelTab{}, (hipStream_t)stream);
}

int mst_stft_mel_f32(const float* x, int32_t B, int32_t L, int32_t n_fft, int32_t hop,
                     int32_t pad_mode, const int32_t* start, const int32_t* len,
                     const int32_t* woff, const float* w, int32_t n_mels, float* out, void* stream) {
  MST_REQUIRE(start && len && woff && w && n_mels > 0 && n_mels <= 128);
  MelTab mt{start, len, woff, w, n_mels};
  return stft_launch(MODE_MEL, x, B, L, n_fft, hop, pad_mode, out, mt, (hipStream_t)stream);
}

int mst_istft_f32(const float* X, int32_t B, int32_t F, int32_t T, int32_t hop, float* y,
                  void* stream) {
  MST_REQUIRE(X && y && B > 0 && F == NB && T > 1 && hop > 0);
  return istft_launch(reinterpret_cast<const float2*>(X), nullptr, nullptr, 0.f, 0, B, T, hop, y,
                      (hipStream_t)stream);
}

// Griffin-Lim runs in clip chunks (clips are independent) so the workspace stays bounded for
// large batches: spectra, windowed frames and signal take ~20 B per bin + 8 KB per frame + 4 B
// per sample. Chunks sized for the 256 MB Infinity Cache (160 MB) were slower than 2 GB ones
// once the iSTFT ran as two passes (config 2: 59.9 vs 52.7 ms): filling the chip with
// workgroups beats cache residency, so the budget is 2 GB (all 256 clips of config 2).
static int gl_chunk(int B, int F, int T, int hop) {
  const size_t per_clip = (size_t)F * T * 20 + (size_t)T * NFFT * 4 + (size_t)hop * (T - 1) * 4;
  static const size_t budget = [] {  // MB; MST_GL_CHUNK_MB overrides (tuning)
    const char* e = getenv("MST_GL_CHUNK_MB");
    return (size_t)(e ? atol(e) : 2048) << 20;
  }();
  size_t cb = budget / (per_clip ? per_clip : 1);
  if (cb < 1) cb = 1;
  return cb < (size_t)B ? (int)cb : B;
}

size_t mst_griffinlim_workspace_size(int32_t B, int32_t F, int32_t T, int32_t hop) {
  if (B <= 0 || F <= 0 || T <= 1 || hop <= 0) return 0;
  const int CB = gl_chunk(B, F, T, hop);
  size_t bins = (size_t)B * F * T, cbins = (size_t)CB * F * T;
  size_t L = (size_t)hop * (T - 1);
  // St (real, all clips) + two complex spectra + two signals + windowed frames of one chunk,
  // each rounded to 256 B
  auto r = [](size_t n) { return (n + 255) / 256 * 256; };
  return r(bins * 4) + 2 * r(cbins * 8) + 2 * r((size_t)CB * L * 4) + r((size_t)CB * T * NFFT * 4);
}

int mst_griffinlim_f32(const float* S, int32_t B, int32_t F, int32_t T, int32_t hop, int32_t n_iter,
                       float momentum, const float* angles0, int32_t mag_from_logpow, float* y,
                       void* workspace, size_t ws_bytes, void* stream) {
  MST_REQUIRE(S && y && workspace && B > 0 && F == NB && T > 1 && hop > 0 && n_iter >= 0);
  MST_REQUIRE(momentum >= 0.f);
  MST_REQUIRE(ws_bytes >= mst_griffinlim_workspace_size(B, F, T, hop));
  MST_REQUIRE(hop * (T - 1) > NFFT / 2);
  hipStream_t st = (hipStream_t)stream;
  auto r = [](size_t n) { return (n + 255) / 256 * 256; };
  const int CB = gl_chunk(B, F, T, hop);
  const size_t bins = (size_t)B * F * T, cbins = (size_t)CB * F * T;
  char* w = (char*)workspace;
  float* St = (float*)w;
  float2* R0 = (float2*)(w + r(bins * 4));
  float2* R1 = (float2*)(w + r(bins * 4) + r(cbins * 8));
  float* sig = (float*)(w + r(bins * 4) + 2 * r(cbins * 8));
  const int L = hop * (T - 1);
  float* sig2 = (float*)(w + r(bins * 4) + 2 * r(cbins * 8) + r((size_t)CB * L * 4));
  float* frames = (float*)((char*)sig2 + r((size_t)CB * L * 4));
  const bool one = gl_one_pass(hop);
  const float beta = momentum / (1.f + momentum);
  // synthesis into `out`; the one-pass kernel also zeroes the seams of `next` (the target after it)
  auto synth = [&](const float2* c, const float2* p, const float* m, int nb, float* out, float* next) {
    return one ? gl_synth_launch(c, p, m, beta, c != nullptr, nb, T, hop, out, next, st)
               : istft2_launch(c, p, m, beta, c != nullptr, nb, T, hop, frames, out, st);
  };
  {
    dim3 grid(ceil_div(T, 32), ceil_div(F, 32), B), block(32, 8);
    hipLaunchKernelGGL(transpose_mag_kernel, grid, block, 0, st, S, F, T, mag_from_logpow, St);
    MST_CHECK_LAUNCH();
  }
  for (int c0 = 0; c0 < B; c0 += CB) {
    const int nb = min(CB, B - c0);
    const float* Sc = St + (size_t)c0 * F * T;
    float* yc = y + (size_t)c0 * L;
    // synthesis targets alternate sig, sig2 and end in the caller's y
    float* outs[2] = {sig, sig2};
    auto target = [&](int it) { return it < n_iter ? outs[it & 1] : yc; };
    if (one) {
      const hipError_t e = hipMemsetAsync(target(0), 0, (size_t)nb * L * 4, st);
      if (e != hipSuccess) return -(int)e;
    }
    // iteration 0 uses the initial phases; iteration 1 has no momentum term (tprev = 0)
    const float2* cur =
        angles0 ? reinterpret_cast<const float2*>(angles0) + (size_t)c0 * F * T : nullptr;
    const float2* prev = nullptr;
    float2* bufs[2] = {R0, R1};
    int rc;
    for (int it = 0; it < n_iter; ++it) {
      rc = synth(cur, prev, Sc, nb, target(it), target(it + 1));
      if (rc) return rc;
      float2* nxt = bufs[it & 1];
      rc = stft_launch(MODE_COMPLEX, target(it), nb, L, NFFT, hop, MST_PAD_REFLECT, (float*)nxt, MelTab{}, st);
      if (rc) return rc;
      prev = (it == 0) ? nullptr : cur;
      cur = nxt;
    }
    rc = synth(cur, prev, Sc, nb, yc, nullptr);
    if (rc) return rc;
  }
  return MST_OK;
}

}  // extern "C"
