// Multi-scale spectral loss (DDSP; README.md:23, stub model/train.py:119-123) with its gradient,
// on gfx950. For each FFT size n in {64 .. 2048} (hop n/4, periodic Hann, center + reflect pad):
//
//   loss_n = mean|S_p - S_t| + alpha * mean|log(S_p + eps) - log(S_t + eps)|,  S = |rfft(frame)|
//   dL/dx  = overlap-add over frames of  w_j * Re sum_f G_f U_f e^{+2 pi i f j / n},
//            G = sign(S_p - S_t)(1 + alpha/(S_p + eps)) / count,  U = X_p / |X_p|
//
// (oracle/spectral_ref.py:multiscale_spectral_loss_grad is the float64 statement.)
//
// Sizes n = 64 .. 1024 run in ONE launch (mss_multi_kernel, grid z = size) and n = 2048 in
// mss_fft2048_kernel (fft.hip). A workgroup owns R = 4096 consecutive samples of one clip's padded
// signal and the frames starting in them, so the gradient is accumulated on chip and written
// once: no atomics, no spectra in HBM. Every frame of pred and of target is transformed on its own as a real FFT (an n/2-point
// complex transform of the even/odd samples plus the post-twist), in place inside one wave;
// the two gradient frames of a frame pair are packed into one Hermitian-completed inverse
// transform (real part = frame a, imaginary part = frame b). The target is transformed once per
// call, in float64 (mss_target_kernel), and the loss kernels read its magnitudes.
// The gradient a workgroup's last three frames put on the 3n/4 samples past its range goes to a
// spill slab (round 5 recomputed those three frames in the next workgroup instead).
// Deterministic: fixed summation order everywhere; each size writes its own gradient and spill
// slabs and mss_sum_kernel adds them in size order; reflect-pad edges are folded in by a final
// kernel.
#include <cstdlib>

#include "common.h"
#include "mss_args.h"

namespace {

constexpr int RWIN = MSS_RWIN;  // padded samples owned per workgroup

// W2048^k = (cos, -sin)(2 pi k / 2048), k < 512, evaluated at compile time (common.h)
struct MssW2048 {
  float2 w[512];
};
constexpr MssW2048 make_mss_w2048() {
  MssW2048 t{};
  double c = 0, s = 0;
  for (int k = 0; k < 512; ++k) {
    cx_sincos_turn(k, 2048, c, s);
    t.w[k] = float2{(float)c, (float)-s};
  }
  return t;
}
__device__ constexpr MssW2048 kMssW2048 = make_mss_w2048();

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
__device__ __forceinline__ c2 conjc(c2 a) { return mk(a.x, -a.y); }

template <bool INV>
__device__ __forceinline__ void dft4(c2& a0, c2& a1, c2& a2, c2& a3) {
  const c2 t0 = a0 + a2, t1 = a0 - a2, t2 = a1 + a3, t3 = a1 - a3;
  const c2 it3 = mk(-t3.y, t3.x);
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

__device__ __forceinline__ int reflect(int i, int L) {
  i = i < 0 ? -i : i;
  return i >= L ? 2 * (L - 1) - i : i;
}

// Every transform runs inside one wave, in place in
// that wave's LDS buffer (a radix-4 stage reads all its inputs into registers, then writes), so
// no workgroup barrier sits inside an FFT. Per round each wave takes 2 FB consecutive frames:
// pass A transforms the FB even ones and keeps their gradient spectra in registers, pass B the
// FB odd ones; the pair-packed Hermitian spectra C = H^a + i H^b then go through one inverse
// transform per pair. After a workgroup barrier every thread adds the round's frames covering
// its RWIN / 256 owned samples (kept in registers) in increasing frame order, so the summation
// order per sample is the frame order, as in the cooperative kernel above.
template <bool INV>
__device__ __forceinline__ c2 twq(const c2* qt, unsigned m, unsigned N) {  // W_N^m, quarter table
  m &= N - 1;
  const unsigned Q = N >> 2, q = m / Q, r = m & (Q - 1);
  const c2 w = qt[r];
  // times (-i)^q by selects (an if/else chain on the per-lane quadrant compiled to divergent
  // branches around each lookup)
  const bool odd = q & 1, neg = q & 2;
  const float a = odd ? w.y : w.x, b = odd ? -w.x : w.y;
  c2 o = mk(neg ? -a : a, neg ? -b : b);
  if (INV) o.y = -o.y;
  return o;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// a W_R^k (INV: a W_R^-k) for a compile-time k < R / 2: exact forms for 1, -+i, (1 -+ i) / sqrt 2
template <int R, bool INV>
__device__ __forceinline__ c2 wconst_f(c2 a, int k) {
  if (k == 0) return a;
  if (4 * k == R) return INV ? mk(-a.y, a.x) : mk(a.y, -a.x);
  constexpr float h = 0.70710678118654752f;
  if (8 * k == R) return INV ? mk(h * (a.x - a.y), h * (a.x + a.y)) : mk(h * (a.x + a.y), h * (a.y - a.x));
  if (8 * k == 3 * R) return INV ? mk(-h * (a.x + a.y), h * (a.x - a.y)) : mk(h * (a.y - a.x), -h * (a.x + a.y));
  const int m = k * (2048 / R), q = m >> 9;  // W2048^m = (-i)^q W2048^(m mod 512), q < 2
  const float2 w = kMssW2048.w[m & 511];
  c2 t = q ? mk(w.y, -w.x) : mk(w.x, w.y);
  if (INV) t.y = -t.y;
  return cmul(a, t);
}

// DFT of R = 2^k points in registers, natural order (radix-2 decimation in time over dft4)
template <int R, bool INV>
__device__ __forceinline__ void dft_f(c2 (&v)[R]) {
  if constexpr (R == 2) {
    const c2 a = v[0], b = v[1];
    v[0] = a + b;
    v[1] = a - b;
  } else if constexpr (R == 4) {
    dft4<INV>(v[0], v[1], v[2], v[3]);
  } else {
    c2 e[R / 2], o[R / 2];
#pragma unroll
    for (int i = 0; i < R / 2; ++i) {
      e[i] = v[2 * i];
      o[i] = v[2 * i + 1];
    }
    dft_f<R / 2, INV>(e);
    dft_f<R / 2, INV>(o);
#pragma unroll
    for (int k = 0; k < R / 2; ++k) {
      const c2 t = wconst_f<R, INV>(o[k], k);
      v[k] = e[k] + t;
      v[k + R / 2] = e[k] - t;
    }
  }
}

// One Stockham radix-R stage of the BWP / M transforms of size M in place in s (Ns = product of
// the earlier radices; qt = the M-point quarter table): every input of the wave is read to
// registers, then written, so no workgroup barrier sits inside an FFT. The twiddle powers are
// formed as w^r = w^(r/2) w^(r - r/2) (at most three products deep).
template <int R, int M, int BWP, int Ns, bool INV>
__device__ __forceinline__ void stage_f(c2* s, const c2* qt, unsigned lane) {
  constexpr int NR = M / R, IT = BWP / R / 64;
  static_assert(IT >= 1, "a stage needs every lane");
  c2 v[IT][R];
  unsigned ln = lane;
  __asm__ volatile("" : "+v"(ln));  // lane-derived addresses formed per stage, not kept live
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const unsigned idx = ln + 64u * it, fr = idx / NR, j = idx % NR;
    const c2* src = s + fr * M + j;
#pragma unroll
    for (int r = 0; r < R; ++r) v[it][r] = src[r * NR];
  }
  wave_sync();
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const unsigned idx = ln + 64u * it, fr = idx / NR, j = idx % NR, k = j & (Ns - 1);
    if constexpr (Ns > 1) {
      c2 w[R];
      w[1] = twq<INV>(qt, k * (M / (R * Ns)), M);
#pragma unroll
      for (int r = 2; r < R; ++r) w[r] = cmul(w[r / 2], w[r - r / 2]);
#pragma unroll
      for (int r = 1; r < R; ++r) v[it][r] = cmul(v[it][r], w[r]);
    }
    dft_f<R, INV>(v[it]);
    c2* d = s + fr * M + (j - k) * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) d[r * Ns] = v[it][r];
  }
  wave_sync();
}

// the stages from Ns on: radix 8 while 8 divides what is left, then the remainder (2 or 4)
template <int M, int BWP, int Ns, bool INV>
__device__ __forceinline__ void stages_f(c2* s, const c2* qt, unsigned lane) {
  if constexpr (Ns < M) {
    constexpr int R = M / Ns < 8 ? M / Ns : 8;
    stage_f<R, M, BWP, Ns, INV>(s, qt, lane);
    stages_f<M, BWP, Ns * R, INV>(s, qt, lane);
  }
}

#ifndef MST_MSS_BW
#define MST_MSS_BW 1024  // complex per wave buffer for n <= MST_MSS_BW (A/B: 512 halves LDS and registers)
#endif
#ifndef MSS_REG_FIRST
#define MSS_REG_FIRST 128  // n/2 from which the forward transform's first stage runs in registers
#endif
#ifndef MST_MSS_OCC
#define MST_MSS_OCC 4  // mss_multi_kernel workgroups per CU (launch bound; LDS allows 4)
#endif
constexpr int MSS_W = 4;  // waves per workgroup
#ifdef MSS_STAMPS  // dev instrumentation (tools/micro/mss_stamps.hip): s_memtime per phase, one size
__device__ unsigned long long g_mss_stamps[2048 * 4 * 4 * 16];
#define MSTAMP(i) do { if (lane == 0 && flat_wg < 2048 && rnd < 4) \
    g_mss_stamps[((flat_wg * 4 + wave) * 4 + rnd) * 16 + (i)] = clock64(); } while (0)
#else
#define MSTAMP(i) do { } while (0)
#endif
template <int LOG2N>
struct MssGeom {
  static constexpr int N = 1 << LOG2N;
  static constexpr int BW = N > MST_MSS_BW ? N : MST_MSS_BW;  // complex per wave buffer
  // LDS bytes: wave buffers, the two quarter tables, the window, the reduction
  static constexpr int LDS = MSS_W * BW * 8 + (N / 4) * 8 + (N / 8) * 8 + N * 4 + 2 * MSS_W * 4;
};
constexpr int MSS_LDS_MAX = MssGeom<10>::LDS;  // the largest size the fused launch serves

// One workgroup (w, b) of size n = 2^LOG2N; lds: MssGeom<LOG2N>::LDS bytes, 16-byte aligned.
template <int LOG2N>
__device__ __forceinline__ void mss_wave_body(const MssArgs& a, int w, int b, char* lds) {
  constexpr int N = 1 << LOG2N, H = N / 4, HALF = N / 2, NBIN = HALF + 1;
  constexpr int W = MSS_W;                   // waves per workgroup
  constexpr int BW = MssGeom<LOG2N>::BW;     // complex per wave buffer
  constexpr int FB = BW / N;                 // transforms per pass
  constexpr int GF = 2 * FB;                 // frames per wave per round
  constexpr int RF = W * GF;                 // frames per round
  constexpr int NE = (FB * NBIN + 63) / 64;  // spectrum entries per lane
  constexpr int OWN = RWIN / 256;            // owned samples per thread
  constexpr int SPILL = (3 * H + 255) / 256;  // per thread: samples past the range its frames reach
  c2* buf = reinterpret_cast<c2*>(lds);                                   // [W * BW]
  c2* qt = buf + W * BW;                                                  // [N / 4]
  c2* qth = qt + N / 4;  // quarter table of the n/2-point forward transforms  [N / 8]
  float* hw = reinterpret_cast<float*>(qth + N / 8);                     // [N]
  float (*red)[W] = reinterpret_cast<float (*)[W]>(hw + N);              // [2][W]

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int L = (int)a.L;
  const float* p = a.pred + (long long)b * a.L;
  const float* tm = a.tmag + (long long)b * a.T * NBIN;  // float64-accurate |X_target| (B, T, NBIN)
  const bool grad = a.dpred != nullptr;
  // twiddles and window from the compile-time W2048 quarter table (N divides 1024): W_N^r =
  // W2048^(r 2048 / N); the periodic Hann in its sin^2 form, sin(pi j / N) = sin(2 pi m / 2048)
  // with m = j 1024 / N < 1024 (the edge values keep their relative precision)
  constexpr int SN = 2048 / N;
  for (int r = tid; r < N / 4; r += 256) {
    const float2 w = kMssW2048.w[r * SN];
    qt[r] = mk(w.x, w.y);
  }
  for (int r = tid; r < N / 8; r += 256) {
    const float2 w = kMssW2048.w[2 * r * SN];
    qth[r] = mk(w.x, w.y);
  }
  for (int j = tid; j < N; j += 256) {
    const int m = j * (SN / 2), q = m >> 9;
    const float2 w = kMssW2048.w[m & 511];
    const float sn = q ? w.x : -w.y;  // sin(2 pi m / 2048): quarter table entry or its cosine
    hw[j] = sn * sn;
  }
  __syncthreads();

  const int own_lo = w * RWIN;
  const int f_own0 = w * (RWIN / H), f_own1 = min(f_own0 + RWIN / H, a.T);
  // Frames [f_own0, f_own1) only: the last three reach 3H samples into the next workgroup's
  // range, and those sums go to a.spill for mss_sum_kernel / mss_fold to add (round 5 recomputed the
  // previous range's last three frames here instead: a nearly empty third round per workgroup).
  const int f_lo = f_own0;
  c2* S = buf + wave * BW;
  float acc[OWN + SPILL];  // sample own_lo + tid + 256 i (i >= OWN: past the range)
#pragma unroll
  for (int i = 0; i < OWN + SPILL; ++i) acc[i] = 0.f;
  float s_abs = 0.f, s_log = 0.f;

#ifdef MSS_STAMPS
  const int flat_wg = w + a.nwg * b;
  int rnd = 0;
#endif
#pragma unroll 1
  for (int t_round = f_lo; t_round < f_own1; t_round += RF) {
    const int t_base = t_round + wave * GF;  // this wave's first frame
    MSTAMP(0);
    if (t_base < f_own1) {                   // wave-uniform
      c2 zga[NE], zgb[NE];
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
        // the target's magnitudes of this pass's frames, loaded ahead of the FFT (the target is
        // transformed once, in float64, by mss_target_kernel: an fp32 transform leaves its
        // near-silent bins at fp32 rounding noise, which log(S + eps) turns into a 1e-3 loss error)
        float stv[NE];
#pragma unroll
        for (int jj = 0; jj < NE; ++jj) {
          const unsigned e = min(lane + 64u * jj, (unsigned)(FB * NBIN - 1)), m = e / NBIN, f = e % NBIN;
          const int t = min(t_base + 2 * (int)m + pass, f_own1 - 1);  // clamped: masked below
          stv[jj] = tm[(long long)t * NBIN + f];
        }
        // load + window FB pred frames t_base + 2m + pass, each an n/2-point complex transform
        // of z_j = w_2j x_2j + i w_2j+1 x_2j+1. Branch-free: a frame past f_own1 loads frame
        // f_own1 - 1 (always in range) and is zeroed by a select; a load under a per-element
        // branch made hipcc wait for each element's loads at the join.
        if constexpr (HALF >= MSS_REG_FIRST) {
          // n >= 256: the first radix-R1 stage runs in registers on the loaded samples (lane
          // element (u, j) takes c = j + r NR1, r < R1) and stores its outputs to the first half
          // of the wave's buffer. Below that, NR1 consecutive pairs per frame are under 128 B and
          // the loads' coalescing cost more than the LDS pass saves (n = 64 / 128 ran 3-6 %
          // slower this way).
          constexpr int R1 = 8, NR1 = HALF / R1, IT1 = BW / 2 / R1 / 64;
          static_assert(IT1 >= 1, "the first stage needs every lane");
#pragma unroll
          for (int it = 0; it < IT1; ++it) {
            const unsigned idx = lane + 64u * it, u = idx / NR1, j = idx % NR1;
            const int t = min(t_base + 2 * (int)u + pass, f_own1 - 1);
            const bool live = t_base + 2 * (int)u + pass < f_own1;
            float x0[R1], x1[R1];
#pragma unroll
            for (int r = 0; r < R1; ++r) {
              const int s0 = t * H + 2 * (int)(j + r * NR1) - HALF;
              x0[r] = p[reflect(s0, L)];
              x1[r] = p[reflect(s0 + 1, L)];
            }
            c2 v[R1];
#pragma unroll
            for (int r = 0; r < R1; ++r) {
              const float2 wj = *reinterpret_cast<const float2*>(hw + 2 * (j + r * NR1));
              v[r] = live ? mk(wj.x * x0[r], wj.y * x1[r]) : mk(0.f, 0.f);
            }
            dft_f<R1, false>(v);
            c2* d = S + u * HALF + j * R1;
#pragma unroll
            for (int r = 0; r < R1; ++r) d[r] = v[r];
          }
          wave_sync();
          MSTAMP(1 + 3 * pass);
          stages_f<HALF, BW / 2, R1, false>(S, qth, lane);
          MSTAMP(2 + 3 * pass);
        } else {
          constexpr int KC = 8;  // elements per load batch (2 KC loads in flight)
#pragma unroll
          for (int k0 = 0; k0 < BW / 128; k0 += KC) {
            float x0[KC], x1[KC];
#pragma unroll
            for (int kk = 0; kk < KC; ++kk) {
              const unsigned e = lane + 64u * (k0 + kk), u = e / HALF, j = e % HALF;
              const int t = min(t_base + 2 * (int)u + pass, f_own1 - 1);
              const int s0 = t * H + 2 * (int)j - HALF;
              x0[kk] = p[reflect(s0, L)];
              x1[kk] = p[reflect(s0 + 1, L)];
            }
#pragma unroll
            for (int kk = 0; kk < KC; ++kk) {
              const unsigned e = lane + 64u * (k0 + kk), u = e / HALF, j = e % HALF;
              const bool live = t_base + 2 * (int)u + pass < f_own1;
              const float2 wj = *reinterpret_cast<const float2*>(hw + 2 * j);
              S[e] = live ? mk(wj.x * x0[kk], wj.y * x1[kk]) : mk(0.f, 0.f);
            }
          }
          wave_sync();
          MSTAMP(1 + 3 * pass);
          stages_f<HALF, BW / 2, 1, false>(S, qth, lane);
          MSTAMP(2 + 3 * pass);
        }
        // spectra, loss, gradient spectra (registers)
#pragma unroll
        for (int jj = 0; jj < NE; ++jj) {
          unsigned ln = lane;
          __asm__ volatile("" : "+v"(ln));  // per-entry indices, not kept live across the loop
          const unsigned e = ln + 64u * jj, m = e / NBIN, f = e % NBIN;
          const int t = t_base + 2 * (int)m + pass;
          c2 zg = mk(0.f, 0.f);
          if (e < FB * NBIN && t < f_own1) {
            // real-FFT post-twist of each signal: X_f = E + W_n^f O, E = (Z_f + conj Z_(n/2-f)) / 2,
            // O = -i (Z_f - conj Z_(n/2-f)) / 2, indices mod n/2
            const c2 wf = twq<false>(qt, f, N);
            const unsigned fa = f & (HALF - 1), fb = (HALF - f) & (HALF - 1);
            const c2 A = S[m * HALF + fa], Bc = conjc(S[m * HALF + fb]);
            const c2 E = (A + Bc) * 0.5f, D = A - Bc;
            const c2 P = E + cmul(wf, mk(D.y * 0.5f, -D.x * 0.5f));
            // hardware sqrt / log2 / rcp (1 ulp): the library forms add ~10 instructions each
            const float sp = __builtin_amdgcn_sqrtf(P.x * P.x + P.y * P.y);
            const float st = stv[jj];
            const float lp = __log2f(sp + a.eps) * 0.69314718055994531f;
            const float lt = __log2f(st + a.eps) * 0.69314718055994531f;
            s_abs += fabsf(sp - st);
            s_log += fabsf(lp - lt);
            if (grad && sp > 0.f) {
              const float sg = sp > st ? 1.f : (sp < st ? -1.f : 0.f);
              const float g = sg * (1.f + a.alpha * __builtin_amdgcn_rcpf(sp + a.eps)) * a.inv_cnt;
              zg = P * (g * __builtin_amdgcn_rcpf(sp));
            }
          }
          if (pass == 0) zga[jj] = zg;
          else zgb[jj] = zg;
        }
        wave_sync();  // every lane has read the spectra before S is overwritten
        MSTAMP(3 + 3 * pass);
      }
      if (grad) {
        // C = H^a + i H^b per pair (H^a_f = Za/2, H^a_{n-f} = conj(Za)/2)
#pragma unroll
        for (int jj = 0; jj < NE; ++jj) {
          unsigned ln = lane;
          __asm__ volatile("" : "+v"(ln));
          const unsigned e = ln + 64u * jj, m = e / NBIN, f = e % NBIN;
          if (e < FB * NBIN) {
            const c2 za = zga[jj], zb = zgb[jj];
            if (f == 0 || f == HALF) {
              S[m * N + f] = mk(za.x, zb.x);
            } else {
              S[m * N + f] = mk(0.5f * (za.x - zb.y), 0.5f * (za.y + zb.x));
              S[m * N + N - f] = mk(0.5f * (za.x + zb.y), 0.5f * (-za.y + zb.x));
            }
          }
        }
        wave_sync();
        stages_f<N, BW, 1, true>(S, qt, lane);
        MSTAMP(7);
      }
    }
    if (!grad) continue;  // uniform over the workgroup: no barrier needed
    __syncthreads();      // every wave's gradient frames are in its buffer
    MSTAMP(8);
    // windowed overlap-add of the round's frames into the owned samples, frames in order. Sample
    // sp is covered by frames th - q (th = sp / H, q = 3 .. 0) at offset sp mod H + q H: four
    // fixed steps, a frame outside the round adding 0 (a per-sample loop had divergent trip
    // counts), over the thread's samples this round's frames reach (a wave-uniform range of i).
    const int r_hi = min(t_round + RF, f_own1);
    const int s_lo = t_round * H - own_lo, s_hi = (r_hi - 1) * H + N - own_lo;
#pragma unroll
    for (int i = 0; i < OWN + SPILL; ++i) {
      if (256 * (i + 1) <= s_lo || 256 * i >= s_hi) continue;
      const unsigned sp = own_lo + tid + 256 * i;  // padded coordinate
      const int th = (int)(sp / H);
      const unsigned jr = sp % H;
      float v = acc[i];
#pragma unroll
      for (int q = 3; q >= 0; --q) {
        const int rel = th - q - t_round;
        const bool ok = rel >= 0 && rel < r_hi - t_round;
        const unsigned rc = ok ? rel : 0u, ww = rc / GF, m = (rc % GF) >> 1, j = jr + q * H;
        const c2 g = buf[ww * BW + m * N + j];
        v = __builtin_fmaf(hw[j], ok ? ((rc & 1) ? g.y : g.x) : 0.f, v);
      }
      acc[i] = v;
    }
    __syncthreads();  // the buffers are read before the next round overwrites them
    MSTAMP(9);
#ifdef MSS_STAMPS
    ++rnd;
#endif
  }

  s_abs = wave_sum(s_abs);
  s_log = wave_sum(s_log);
  if (lane == 0) {
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
  // this size's gradient slab (the sizes are summed in order by mss_sum_kernel)
  float* dp = a.dpred + (long long)b * a.L;
  float* ed = a.edges + (long long)b * N;
  const int own_hi = min(own_lo + RWIN, L + N);
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
  for (int i = 0; i < SPILL; ++i) {
    const int o = tid + 256 * i;
    if (o < 3 * H) spl[o] = acc[OWN + i];
  }
}

// ------------------------------------------------------------------ target magnitudes, float64
// |STFT_n(target)| for every size, frame-major (B, T_n, n/2 + 1): the transform and the power in
// float64, the power rounded to float and its square root taken in float: an fp32 transform leaves bins far below the frame's peak at fp32 rounding noise (a
// silent or decaying target's high bins), and log(S + 1e-7) turns that noise into a 1e-3 loss
// error against the float64 definition (bench_aux's silent piano pair). The target needs no
// gradient, so it is transformed once per call here and the loss kernels read its magnitudes.
// One wave transforms FBT = BWT / (n/2) frames at a time in its LDS buffer (n/2-point complex
// Stockham FFT of z_j = w_2j x_2j + i w_2j+1 x_2j+1, then the real-FFT post-twist), twiddles
// from a compile-time float64 W2048 table.
struct MssW2048d {
  double2 w[512];
};
constexpr MssW2048d make_mss_w2048d() {
  MssW2048d t{};
  double c = 0, s = 0;
  for (int k = 0; k < 512; ++k) {
    cx_sincos_turn(k, 2048, c, s);
    t.w[k] = double2{c, -s};
  }
  return t;
}
__device__ constexpr MssW2048d kMssW2048d = make_mss_w2048d();

struct d2 {
  double x, y;
};
__device__ __forceinline__ d2 dk(double x, double y) { return d2{x, y}; }
__device__ __forceinline__ d2 operator+(d2 a, d2 b) { return dk(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ d2 operator-(d2 a, d2 b) { return dk(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ d2 dmul(d2 a, d2 b) { return dk(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }

// W_N^m (N | 2048) from the quarter table: W2048^(m 2048 / N) = (-i)^q W2048^r
__device__ __forceinline__ d2 twd(const d2* qt, int m, int N) {
  const int k = (m & (N - 1)) * (2048 / N), q = k >> 9, r = k & 511;
  const d2 w = qt[r];
  const bool odd = q & 1, neg = q & 2;
  const double a = odd ? w.y : w.x, b = odd ? -w.x : w.y;
  return dk(neg ? -a : a, neg ? -b : b);
}

// LDS slot of complex element i of a wave buffer: i ^ ((i >> 3) & 15) ^ ((i >> 6) & 15) (bits 3..9
// into bits 0..3; bits 6 and up stay, so bit 3 and then bits 0..2 are recoverable: a bijection).
// Chosen with the bank model of tools/lds_swizzle_search.py (radix8 mode: ds_read_b128 16-lane
// groups {0-3,12-15,20-27} / {4-11,16-19,28-31}, 16 slots per 256-B row; ds_write_b128 8
// contiguous lanes, 8 slots per 128-B row) over every access of the register-first radix-8
// schedule below at n = 64 .. 2048: 1058 modelled conflict cycles over 372 LDS instructions per
// wave pass of every size (1174 for one shift-XOR term, 956 for a searched 8-bit XOR map that
// costs ~24 VALU per address instead of 5; the round-5 radix-4 schedule: 1004 over 644).
// Linear: tsw(a | b) = tsw(a) ^ tsw(b) for disjoint bits, so the loops form one lane-dependent
// slot and XOR compile-time constants into it.
__device__ __forceinline__ constexpr int tsw(int i) { return i ^ ((i >> 3) & 15) ^ ((i >> 6) & 15); }

// a W_R^k for a compile-time k < R / 2 (R | 16): exact forms for 1, -i and (+-1 - i) / sqrt 2
template <int R>
__device__ __forceinline__ d2 wconst(d2 a, int k) {
  if (k == 0) return a;
  if (4 * k == R) return dk(a.y, -a.x);
  constexpr double h = 0.70710678118654752440;
  if (8 * k == R) return dk(h * (a.x + a.y), h * (a.y - a.x));
  if (8 * k == 3 * R) return dk(h * (a.y - a.x), -h * (a.x + a.y));
  const int m = k * (2048 / R), q = m >> 9;  // W2048^m = (-i)^q W2048^(m mod 512)
  const double2 w = kMssW2048d.w[m & 511];
  const d2 t = q ? dk(w.y, -w.x) : dk(w.x, w.y);
  return dmul(a, t);
}

// W_R^r = (cos, -sin)(2 pi r / R) for a compile-time r < R (R | 2048), from the float64 table
template <int R>
__device__ __forceinline__ d2 wturn(int r) {
  const int m = r * (2048 / R), q = m >> 9;  // W2048^m = (-i)^q W2048^(m mod 512)
  const double2 w = kMssW2048d.w[m & 511];
  const double a = (q & 1) ? w.y : w.x, b = (q & 1) ? -w.x : w.y;
  return (q & 2) ? dk(-a, -b) : dk(a, b);
}

// forward DFT of R = 2^k points in registers, natural order (radix-2 decimation in time)
template <int R>
__device__ __forceinline__ void dft_d(d2 (&v)[R]) {
  if constexpr (R == 1) {
    return;
  } else if constexpr (R == 2) {
    const d2 a = v[0], b = v[1];
    v[0] = a + b;
    v[1] = a - b;
  } else {
    d2 e[R / 2], o[R / 2];
#pragma unroll
    for (int i = 0; i < R / 2; ++i) {
      e[i] = v[2 * i];
      o[i] = v[2 * i + 1];
    }
    dft_d<R / 2>(e);
    dft_d<R / 2>(o);
#pragma unroll
    for (int k = 0; k < R / 2; ++k) {
      const d2 t = wconst<R>(o[k], k);
      v[k] = e[k] + t;
      v[k + R / 2] = e[k] - t;
    }
  }
}

// One Stockham radix-R stage of the BWT / M transforms of size M in place in s (Ns = product of
// the earlier stages' radices): every input of the wave read to registers, then written
template <int R, int M, int BWT, int Ns>
__device__ __forceinline__ void stage_d(d2* s, const d2* qt, int lane) {
  constexpr int NR = M / R, IT = BWT / R / 64;
  static_assert(IT >= 1, "a stage needs every lane");
  d2 v[IT][R];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = lane + 64 * it, fr = idx / NR, j = idx - fr * NR;
    const int pb = tsw(fr * M + j);
#pragma unroll
    for (int r = 0; r < R; ++r) v[it][r] = s[pb ^ tsw(r * NR)];
  }
  wave_sync();
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = lane + 64 * it, fr = idx / NR, j = idx - fr * NR, k = j & (Ns - 1);
    const d2 w1 = twd(qt, k, Ns * R);
    d2 w = w1;
#pragma unroll
    for (int r = 1; r < R; ++r) {
      v[it][r] = dmul(v[it][r], w);
      if (r + 1 < R) w = dmul(w, w1);
    }
    dft_d<R>(v[it]);
    const int pb = tsw(fr * M + (j - k) * R + k);
#pragma unroll
    for (int r = 0; r < R; ++r) s[pb ^ tsw(r * Ns)] = v[it][r];
  }
  wave_sync();
}

// the stages after the first: radix 8 while 8 divides what is left, then the remainder (2 or 4)
template <int M, int BWT, int Ns>
__device__ __forceinline__ void stages_d(d2* s, const d2* qt, int lane) {
  if constexpr (Ns < M) {
    constexpr int R = M / Ns < 8 ? M / Ns : 8;
    stage_d<R, M, BWT, Ns>(s, qt, lane);
    stages_d<M, BWT, Ns * R>(s, qt, lane);
  }
}

#ifndef MSS_R16
#define MSS_R16 1  // n = 2048: a radix-16 first stage (5 VGPRs spilled; radix 8 spills 38)
#endif
constexpr int MSS_TW = 4;           // waves per target workgroup
constexpr int MSS_TBW = 512;        // complex doubles per wave buffer (n/2 <= 512); n = 2048: 1024
constexpr int MSS_TROUNDS = 4;      // frame batches per wave per workgroup
// LDS: wave buffers + the twiddle table; n <= 1024 (40 KB, three workgroups per CU) and n = 2048
// (72 KB, two) run as separate launches so the small sizes are not held to the large size's LDS
template <bool BIG>
constexpr int mss_tlds() { return MSS_TW * (BIG ? 1024 : 512) * 16 + 512 * 16; }

struct MssTgt {
  const float* target;
  long long L;
  int nsz;
  int lg[8], T[8], nblk[8];
  float* tmag[8];
};

template <int LOG2N>
__device__ __forceinline__ void mss_target_body(const MssTgt& A, int z, int blk, int b, char* lds) {
  constexpr int N = 1 << LOG2N, H = N / 4, HALF = N / 2, NBIN = HALF + 1;
  constexpr int BWT = HALF > MSS_TBW ? HALF : MSS_TBW;
  constexpr int FBT = BWT / HALF;            // frames per wave batch
  constexpr int NEO = (FBT * NBIN + 63) / 64;  // output bins per lane
  d2* qt = reinterpret_cast<d2*>(lds);
  d2* S = qt + 512 + (threadIdx.x >> 6) * BWT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int r = threadIdx.x; r < 512; r += 256) {
    const double2 w = kMssW2048d.w[r];
    qt[r] = dk(w.x, w.y);
  }
  __syncthreads();
  const int L = (int)A.L, T = A.T[z];
  const float* x = A.target + (long long)b * A.L;
  float* out = A.tmag[z] + (long long)b * T * NBIN;
  constexpr int PER_WG = MSS_TW * FBT * MSS_TROUNDS;
  // The first FFT stage runs on the loaded samples in registers (no LDS pass for the load):
  // radix R1 over the FBT frames' z_j = w_2j x_2j + i w_2j+1 x_2j+1 (periodic Hann in float64,
  // reflect pad), lane element (u, j) takes c = j + r NR1, r < R1. The window's angles there are
  // 2 pi (2j + {0, 1}) / N + 2 pi r / R1: the lane keeps cos / sin of its two base angles and
  // rotates them by compile-time constants (float64 angle sums, no table reads per batch).
  constexpr int R1 = (MSS_R16 && BWT >= 1024 && HALF >= 1024) ? 16 : (HALF < 8 ? HALF : 8);
  constexpr int NR1 = HALF / R1, IT1 = BWT / R1 / 64;
  static_assert(IT1 >= 1, "the first stage needs every lane");
  double ca[IT1], sa[IT1], cb[IT1], sb[IT1];
#pragma unroll
  for (int it = 0; it < IT1; ++it) {
    const int j = (lane + 64 * it) % NR1;
    const d2 p = twd(qt, 2 * j, N), q = twd(qt, 2 * j + 1, N);  // W_N^k = (cos, -sin)(2 pi k / N)
    ca[it] = p.x;
    sa[it] = -p.y;
    cb[it] = q.x;
    sb[it] = -q.y;
  }
#pragma unroll 1
  for (int rd = 0; rd < MSS_TROUNDS; ++rd) {
    const int t0 = blk * PER_WG + (rd * MSS_TW + wave) * FBT;  // this wave's first frame
    if (t0 >= T) break;                                        // wave-uniform
    // every sample of the batch is loaded before any is used (BWT / 64 pairs per lane in flight)
    float xa[IT1][R1], xb[IT1][R1];
#pragma unroll
    for (int it = 0; it < IT1; ++it) {
      const int idx = lane + 64 * it, u = idx / NR1, j = idx - u * NR1;
      const int t = min(t0 + u, T - 1);
#pragma unroll
      for (int r = 0; r < R1; ++r) {
        const int s0 = t * H + 2 * (j + r * NR1) - HALF;
        xa[it][r] = x[reflect(s0, L)];
        xb[it][r] = x[reflect(s0 + 1, L)];
      }
    }
#pragma unroll
    for (int it = 0; it < IT1; ++it) {
      const int idx = lane + 64 * it, u = idx / NR1, j = idx - u * NR1;
      d2 v[R1];
#pragma unroll
      for (int r = 0; r < R1; ++r) {
        const d2 rot = wturn<R1>(r);  // (cos, -sin)(2 pi r / R1), compile-time
        const double wa = 0.5 - 0.5 * (ca[it] * rot.x + sa[it] * rot.y);
        const double wb = 0.5 - 0.5 * (cb[it] * rot.x + sb[it] * rot.y);
        v[r] = dk(wa * (double)xa[it][r], wb * (double)xb[it][r]);
      }
      dft_d<R1>(v);
      const int pb = tsw(u * HALF + j * R1);
#pragma unroll
      for (int r = 0; r < R1; ++r) S[pb ^ tsw(r)] = v[r];
    }
    wave_sync();
    stages_d<HALF, BWT, R1>(S, qt, lane);
    // post-twist X_f = E + W_N^f O, E = (Z_f + conj Z_(n/2-f)) / 2, O = -i (Z_f - conj Z_(n/2-f)) / 2
#pragma unroll
    for (int jj = 0; jj < NEO; ++jj) {
      const int e = lane + 64 * jj, m = e / NBIN, f = e - m * NBIN;
      const int t = t0 + m;
      if (e < FBT * NBIN && t < T) {
        const d2 Af = S[tsw(m * HALF + (f & (HALF - 1)))], Bf = S[tsw(m * HALF + ((HALF - f) & (HALF - 1)))];
        const d2 E = dk(0.5 * (Af.x + Bf.x), 0.5 * (Af.y - Bf.y));
        const d2 D = dk(0.5 * (Af.y + Bf.y), -0.5 * (Af.x - Bf.x));  // -i (A - conj B) / 2
        const d2 X = E + dmul(twd(qt, f, N), D);
        // |X| from the float64 power rounded to float, by the hardware square root (1 ulp; the
        // correctly rounded float64 sqrt is ~15 instructions at the float64 rate)
        out[(long long)t * NBIN + f] = __builtin_amdgcn_sqrtf((float)(X.x * X.x + X.y * X.y));
      }
    }
    wave_sync();  // the spectra are read before the next batch overwrites the buffer
  }
}

// grid (max nblk, B, sizes of the launch): n = 64 .. 1024 in one launch, n = 2048 in another
__global__ __launch_bounds__(256, 3) void mss_target_kernel(const MssTgt A) {
  __shared__ __attribute__((aligned(16))) char lds[mss_tlds<false>()];
  const int z = blockIdx.z, blk = blockIdx.x, b = blockIdx.y;
  if (blk >= A.nblk[z]) return;
  switch (A.lg[z]) {
    case 6: mss_target_body<6>(A, z, blk, b, lds); break;
    case 7: mss_target_body<7>(A, z, blk, b, lds); break;
    case 8: mss_target_body<8>(A, z, blk, b, lds); break;
    case 9: mss_target_body<9>(A, z, blk, b, lds); break;
    default: mss_target_body<10>(A, z, blk, b, lds); break;
  }
}
__global__ __launch_bounds__(256, 2) void mss_target2048_kernel(const MssTgt A) {
  __shared__ __attribute__((aligned(16))) char lds[mss_tlds<true>()];
  const int blk = blockIdx.x, b = blockIdx.y;
  if (blk >= A.nblk[0]) return;
  mss_target_body<11>(A, 0, blk, b, lds);
}

int mss_target_frames_per_wg(int lg) {
  const int half = 1 << (lg - 1);
  const int bwt = half > MSS_TBW ? half : MSS_TBW;
  return MSS_TW * (bwt / half) * MSS_TROUNDS;
}

// Sizes n = 64 .. 1024 of one loss call in ONE launch: blockIdx.z picks the size (its workgroups
// are (w < nwg, b)), so the per-size grids (1.7 residency waves each at config 5) no longer end in
// a partial wave apiece and no launch gap separates the sizes. Every size writes its own gradient
// slab; mss_sum_kernel adds them in size order (the order the per-size launches accumulated in).
struct MssMulti {
  MssArgs s[8];
  int lg[8];
  int nsz;
};

__global__ __launch_bounds__(256, MST_MSS_OCC) void mss_multi_kernel(const MssMulti m) {
  __shared__ __attribute__((aligned(16))) char lds[MSS_LDS_MAX];
  const int z = blockIdx.z;
  const MssArgs& a = m.s[z];
  const int w = blockIdx.x, b = blockIdx.y;
  if (w >= a.nwg) return;  // whole workgroup, before any barrier
  switch (m.lg[z]) {
    case 6: mss_wave_body<6>(a, w, b, lds); break;
    case 7: mss_wave_body<7>(a, w, b, lds); break;
    case 8: mss_wave_body<8>(a, w, b, lds); break;
    case 9: mss_wave_body<9>(a, w, b, lds); break;
    default: mss_wave_body<10>(a, w, b, lds); break;
  }
}

// The gradient a workgroup's last three frames put on the 3n/4 padded samples past its range
// (MssArgs::spill): the value for padded sample pp of clip b, or 0 where no workgroup spills.
__device__ __forceinline__ float spill_at(const float* sp, int nwg, int hs, long long b, long long pp) {
  const long long w = pp / MSS_RWIN;
  const int o = (int)(pp - w * MSS_RWIN);
  return (w >= 1 && w < nwg && o < hs) ? sp[(b * nwg + w - 1) * hs + o] : 0.f;
}

// dpred[b, x] = sum over sizes in call order (the per-size launches' order) of that size's slab
// plus the spill from the previous workgroup's range (spill_at). Grid (blocks, B): one clip row
// per blockIdx.y. vec: L % 4 == 0 and dpred 16-byte aligned (the slabs are, stride a multiple of
// 4); a 4-sample group never straddles a spill boundary (MSS_RWIN, n / 2 and 3n / 4 are multiples
// of 4).
struct SumArgs {
  const float* slabs;  // size s's slab at slabs + s * stride, (B, L) each
  long long stride, L;
  int nsz, vec;
  float* dpred;
  const float* spill[8];
  int half[8], hs[8], nwg[8];
};

__global__ __launch_bounds__(256) void mss_sum_kernel(const SumArgs a) {
  const long long b = blockIdx.y, L = a.L;
  float* dp = a.dpred + b * L;
  const long long step = (long long)gridDim.x * blockDim.x;
  if (a.vec) {
    for (long long x = 4 * ((long long)blockIdx.x * blockDim.x + threadIdx.x); x < L; x += 4 * step) {
      f32x4 v;
      for (int s = 0; s < a.nsz; ++s) {
        f32x4 t = *reinterpret_cast<const f32x4*>(a.slabs + s * a.stride + b * L + x);
        const long long pp = x + a.half[s], w = pp / MSS_RWIN;
        const int o = (int)(pp - w * MSS_RWIN);
        if (w >= 1 && w < a.nwg[s] && o < a.hs[s])
          t += *reinterpret_cast<const f32x4*>(a.spill[s] + (b * a.nwg[s] + w - 1) * a.hs[s] + o);
        v = s == 0 ? t : v + t;
      }
      *reinterpret_cast<f32x4*>(dp + x) = v;
    }
    return;
  }
  for (long long x = (long long)blockIdx.x * blockDim.x + threadIdx.x; x < L; x += step) {
    float v = 0.f;
    for (int s = 0; s < a.nsz; ++s) {
      const float t = a.slabs[s * a.stride + b * L + x] + spill_at(a.spill[s], a.nwg[s], a.hs[s], b, x + a.half[s]);
      v = s == 0 ? t : v + t;
    }
    dp[x] = v;
  }
}

// dpred += reflect-pad edge gradients of every size (in size order: deterministic).
struct FoldArgs {
  float* dpred;
  const float* edges;  // concatenated per size: (B, n_s)
  long long L;
  int B, nsz;
  int n[8];
  long long off[8];
  const float* spill[8];  // the tail-pad samples' spill (spill_at), by size
  int nwg[8];
};

__device__ void mss_fold(const FoldArgs& a, int b) {
  const int L = (int)a.L;
  float* dp = a.dpred + (long long)b * a.L;
  int maxhalf = 0;
  for (int s = 0; s < a.nsz; ++s) maxhalf = max(maxhalf, a.n[s] / 2);
  // head: padded p < n/2 is x[n/2 - p]; tail: x[2(L-1) - (L + k)] = x[L - 2 - k]
  if (L > 2 * maxhalf + 1) {
    // head targets [1, maxhalf] and tail targets [L - 1 - maxhalf, L - 2] are disjoint: one
    // read-modify-write per target, the sizes added in size order as below (same sums)
    for (int i = threadIdx.x; i < maxhalf; i += blockDim.x) {
      const int h = i + 1;
      float vh = dp[h], vt = dp[L - 2 - i];
      for (int s = 0; s < a.nsz; ++s) {
        const int half = a.n[s] / 2;
        const float* ed = a.edges + a.off[s] + (long long)b * a.n[s];
        if (h <= half) vh += ed[half - h];
        if (i < half) vt += ed[half + i] + spill_at(a.spill[s], a.nwg[s], 3 * a.n[s] / 4, b, a.L + half + i);
      }
      dp[h] = vh;
      dp[L - 2 - i] = vt;
    }
    return;
  }
  for (int s = 0; s < a.nsz; ++s) {  // short clips: head and tail overlap
    const int n = a.n[s], half = n / 2;
    const float* ed = a.edges + a.off[s] + (long long)b * n;
    for (int k = threadIdx.x; k < half; k += blockDim.x) dp[half - k] += ed[k];
    __syncthreads();
    for (int k = threadIdx.x; k < half; k += blockDim.x)
      dp[L - 2 - k] += ed[half + k] + spill_at(a.spill[s], a.nwg[s], 3 * n / 4, b, a.L + half + k);
    __syncthreads();
  }
}

struct LossArgs {
  const float* partial;
  long long off[8];
  int cnt[8];  // B * nwg per size
  float inv_cnt[8];
  int nsz;
  float alpha;
  float* loss;
};

__device__ void mss_loss(const LossArgs& a) {
  __shared__ double red[4];
  double tot = 0.0;
  constexpr int U = 8;  // partial pairs in flight per thread (clamped loads, masked adds)
  for (int s = 0; s < a.nsz; ++s) {
    double sa = 0.0, sl = 0.0;
    const int cnt = a.cnt[s];
    const float2* part = reinterpret_cast<const float2*>(a.partial + a.off[s]);
    for (int i0 = threadIdx.x; i0 < cnt; i0 += U * blockDim.x) {
      float2 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = part[min(i0 + u * (int)blockDim.x, cnt - 1)];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (i0 + u * (int)blockDim.x < cnt) {
          sa += v[u].x;
          sl += v[u].y;
        }
      }
    }
    tot += (sa + (double)a.alpha * sl) * (double)a.inv_cnt[s];
  }
  tot = wave_sum_d(tot);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = tot;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < (int)(blockDim.x / 64); ++i) t += red[i];
    a.loss[0] = (float)t;
  }
}

// One launch after the per-size kernels: blocks 0 .. B-1 fold the edge gradients of clip b,
// the last block reduces the loss partials.
struct FinishArgs {
  FoldArgs f;
  LossArgs l;
  int fold_blocks;
};

__global__ __launch_bounds__(256) void mss_finish_kernel(const FinishArgs a) {
  if ((int)blockIdx.x < a.fold_blocks) mss_fold(a.f, blockIdx.x);
  else mss_loss(a.l);
}

int log2i(int n) {
  int l = 0;
  while ((1 << l) < n) ++l;
  return (1 << l) == n ? l : -1;
}

struct Plan {
  int nsz;
  int n[8], T[8], nwg[8];
  long long part_off[8], edge_off[8], slab_off[8], slab_stride, tmag_off[8], spill_off[8];
  size_t bytes;
};

int make_plan(int64_t B, int64_t L, int32_t n_sizes, const int32_t* sizes, Plan& pl) {
  if (B <= 0 || L <= 0 || n_sizes <= 0 || n_sizes > 8 || sizes == nullptr) return MST_EINVAL;
  if (L >= (1ll << 30)) return MST_EINVAL;
  pl.nsz = n_sizes;
  long long part = 0, edge = 0;
  for (int s = 0; s < n_sizes; ++s) {
    const int n = sizes[s], lg = log2i(n);
    if (lg < 6 || lg > 11 || L <= n / 2) return MST_EINVAL;
    pl.n[s] = n;
    pl.T[s] = (int)(1 + L / (n / 4));
    pl.nwg[s] = ceil_div(L + n, RWIN);
    pl.part_off[s] = part;
    part += B * pl.nwg[s] * 2;
    pl.edge_off[s] = edge;
    edge += B * n;
  }
  // per-size gradient slabs (B, L), summed in size order by mss_sum_kernel
  pl.slab_stride = (B * L + 3) / 4 * 4;
  const long long slab0 = (part + edge + 3) / 4 * 4;
  for (int s = 0; s < n_sizes; ++s) pl.slab_off[s] = slab0 + s * pl.slab_stride;
  // the target's float64-accurate magnitudes per size (B, T_n, n/2 + 1), 16-byte aligned
  long long tm = slab0 + n_sizes * pl.slab_stride;
  for (int s = 0; s < n_sizes; ++s) {
    pl.tmag_off[s] = tm;
    tm += (B * pl.T[s] * (pl.n[s] / 2 + 1) + 3) / 4 * 4;
  }
  // the gradient past each workgroup's range per size (B, nwg, 3n/4)
  for (int s = 0; s < n_sizes; ++s) {
    pl.spill_off[s] = tm;
    tm += B * pl.nwg[s] * (3 * pl.n[s] / 4);
  }
  pl.bytes = (size_t)tm * sizeof(float);
  for (int s = 0; s < n_sizes; ++s) pl.edge_off[s] += part;
  return 0;
}

}  // namespace

extern "C" {

size_t mst_mss_workspace_size(int64_t B, int64_t L, int32_t n_sizes, const int32_t* sizes) {
  Plan pl;
  if (make_plan(B, L, n_sizes, sizes, pl) != 0) return 0;
  return pl.bytes;
}

int mst_mss_loss_f32(const float* pred, const float* target, int64_t B, int64_t L,
                     int32_t n_sizes, const int32_t* sizes, float alpha, float eps, float* loss,
                     float* dpred, void* ws, size_t ws_bytes, void* stream) {
  Plan pl;
  const int rc = make_plan(B, L, n_sizes, sizes, pl);
  if (rc != 0) return rc;
  MST_REQUIRE(pred && target && loss && ws && ws_bytes >= pl.bytes && B <= 65535);
  hipStream_t st = (hipStream_t)stream;
  float* w = (float*)ws;
  MST_REQUIRE(((uintptr_t)ws & 15) == 0);
  // the target's magnitudes: n = 64 .. 1024 in one launch, n = 2048 in another
  MssTgt tg[2];
  unsigned max_blk[2] = {0, 0};
  for (int k = 0; k < 2; ++k) {
    tg[k].target = target;
    tg[k].L = L;
    tg[k].nsz = 0;
  }
  for (int s = 0; s < pl.nsz; ++s) {
    const int lg = log2i(pl.n[s]), k = lg == 11 ? 1 : 0, z = tg[k].nsz++;
    tg[k].lg[z] = lg;
    tg[k].T[z] = pl.T[s];
    tg[k].nblk[z] = ceil_div(pl.T[s], mss_target_frames_per_wg(lg));
    tg[k].tmag[z] = w + pl.tmag_off[s];
    max_blk[k] = max_blk[k] > (unsigned)tg[k].nblk[z] ? max_blk[k] : (unsigned)tg[k].nblk[z];
  }
  if (tg[0].nsz > 0) {
    hipLaunchKernelGGL(mss_target_kernel, dim3(max_blk[0], (unsigned)B, (unsigned)tg[0].nsz), dim3(256), 0, st, tg[0]);
    MST_CHECK_LAUNCH();
  }
  if (tg[1].nsz > 0) {
    hipLaunchKernelGGL(mss_target2048_kernel, dim3(max_blk[1], (unsigned)B, 1), dim3(256), 0, st, tg[1]);
    MST_CHECK_LAUNCH();
  }
  MssMulti mm;
  mm.nsz = 0;
  unsigned max_nwg = 0;
  for (int s = 0; s < pl.nsz; ++s) {
    MssArgs a;
    a.pred = pred;
    a.target = target;
    a.tmag = w + pl.tmag_off[s];
    a.L = L;
    a.T = pl.T[s];
    a.nwg = pl.nwg[s];
    a.alpha = alpha;
    a.eps = eps;
    a.inv_cnt = (float)(1.0 / ((double)B * pl.T[s] * (pl.n[s] / 2 + 1)));
    a.dpred = dpred ? w + pl.slab_off[s] : nullptr;  // this size's slab
    a.edges = w + pl.edge_off[s];
    a.partial = w + pl.part_off[s];
    a.spill = w + pl.spill_off[s];
    const int lg = log2i(pl.n[s]);
    if (lg == 11) {  // register-resident fft1024_v2 kernel (fft.hip)
      mss_fft2048_launch(a, (unsigned)pl.nwg[s], (unsigned)B, st);
      MST_CHECK_LAUNCH();
    } else {
      mm.s[mm.nsz] = a;
      mm.lg[mm.nsz] = lg;
      ++mm.nsz;
      max_nwg = max_nwg > (unsigned)pl.nwg[s] ? max_nwg : (unsigned)pl.nwg[s];
    }
  }
  if (mm.nsz > 0) {
    hipLaunchKernelGGL(mss_multi_kernel, dim3(max_nwg, (unsigned)B, (unsigned)mm.nsz), dim3(256), 0, st, mm);
    MST_CHECK_LAUNCH();
  }
  if (dpred) {
    SumArgs sa;
    sa.slabs = w + pl.slab_off[0];
    sa.stride = pl.slab_stride;
    sa.L = L;
    sa.nsz = pl.nsz;
    sa.vec = (L % 4 == 0 && ((uintptr_t)dpred & 15) == 0) ? 1 : 0;
    sa.dpred = dpred;
    for (int s = 0; s < pl.nsz; ++s) {
      sa.spill[s] = w + pl.spill_off[s];
      sa.half[s] = pl.n[s] / 2;
      sa.hs[s] = 3 * pl.n[s] / 4;
      sa.nwg[s] = pl.nwg[s];
    }
    const long long per = sa.vec ? (L + 3) / 4 : L;
    const long long blocks = (per + 255) / 256;
    hipLaunchKernelGGL(mss_sum_kernel, dim3((unsigned)(blocks < 1024 ? blocks : 1024), (unsigned)B), dim3(256), 0, st, sa);
    MST_CHECK_LAUNCH();
  }
  FinishArgs fa;
  fa.fold_blocks = dpred ? (int)B : 0;
  FoldArgs& f = fa.f;
  f.dpred = dpred;
  f.edges = w;
  f.L = L;
  f.B = (int)B;
  f.nsz = pl.nsz;
  LossArgs& la = fa.l;
  la.partial = w;
  la.nsz = pl.nsz;
  la.alpha = alpha;
  la.loss = loss;
  for (int s = 0; s < pl.nsz; ++s) {
    f.n[s] = pl.n[s];
    f.off[s] = pl.edge_off[s];
    f.spill[s] = w + pl.spill_off[s];
    f.nwg[s] = pl.nwg[s];
    la.off[s] = pl.part_off[s];
    la.cnt[s] = (int)(B * pl.nwg[s]);
    la.inv_cnt[s] = (float)(1.0 / ((double)B * pl.T[s] * (pl.n[s] / 2 + 1)));
  }
  mss_finish_kernel<<<(unsigned)(fa.fold_blocks + 1), 256, 0, st>>>(fa);
  MST_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
