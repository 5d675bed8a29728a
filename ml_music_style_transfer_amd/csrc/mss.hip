// Multi-scale spectral loss (DDSP; README.md:23, stub model/train.py:119-123) with its gradient,
// on gfx950. For each FFT size n in {64 .. 2048} (hop n/4, periodic Hann, center + reflect pad):
//
//   loss_n = mean|S_p - S_t| + alpha * mean|log(S_p + eps) - log(S_t + eps)|,  S = |rfft(frame)|
//   dL/dx  = overlap-add over frames of  w_j * Re sum_f G_f U_f e^{+2 pi i f j / n},
//            G = sign(S_p - S_t)(1 + alpha/(S_p + eps)) / count,  U = X_p / |X_p|
//
// (oracle/spectral_ref.py:multiscale_spectral_loss_grad is the float64 statement.)
//
// One launch per size. A workgroup owns R = 4096 consecutive samples of one clip's padded
// signal and computes every frame that overlaps them (3 halo frames recomputed at the left
// edge), so the gradient is accumulated in LDS and written once: no atomics, no spectra in
// HBM. Per frame the two real signals are packed as one complex signal z = w (p + i q) and
// transformed together (P_f = (Z_f + conj Z_{n-f})/2, Q_f = (Z_f - conj Z_{n-f})/2i); the two
// gradient frames of a frame pair are likewise packed into one Hermitian-completed inverse
// transform (real part = frame a, imaginary part = frame b). The FFTs are Stockham radix-4
// (+ one radix-2 stage for odd log2 n) over LDS, 2048 complex per chunk of frames.
// Deterministic: fixed summation order everywhere; per-size launches accumulate into dpred
// in stream order, reflect-pad edges are folded in by a final kernel.
#include <cstdlib>

#include "common.h"
#include "mss_args.h"

namespace {

constexpr int RWIN = MSS_RWIN;  // padded samples owned per workgroup
constexpr int CAP = 2048;    // complex values per LDS FFT buffer
#ifndef MSS_NT
#define MSS_NT 256
#endif
constexpr int NT = MSS_NT;  // threads per workgroup

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

// exp(-+2 pi i m / n) from a quarter-wave table qt[r] = (cos, -sin)(2 pi r / n), r < n/4.
template <int LOG2N, bool INV>
__device__ __forceinline__ c2 twid(const c2* qt, int m) {
  constexpr int N = 1 << LOG2N, Q = N / 4;
  m &= N - 1;
  const int q = m / Q, r = m & (Q - 1);
  const c2 w = qt[r];
  c2 o;
  if (q == 0) o = w;
  else if (q == 1) o = mk(w.y, -w.x);
  else if (q == 2) o = mk(-w.x, -w.y);
  else o = mk(-w.y, w.x);
  if (INV) o.y = -o.y;
  return o;
}

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

// One Stockham stage (radix R, Ns = product of earlier radices) on `frames` transforms.
template <int LOG2N, int R, bool INV>
__device__ __forceinline__ void stage(const c2* src, c2* dst, int Ns, int frames, const c2* qt) {
  constexpr int N = 1 << LOG2N, NR = N / R;
  const int total = frames * NR;
  for (int idx = threadIdx.x; idx < total; idx += NT) {
    const int fr = idx / NR, j = idx - fr * NR;
    const c2* s = src + fr * N;
    c2* d = dst + fr * N;
    const int k = j & (Ns - 1);
    const int step = N / (Ns * R);
    if constexpr (R == 4) {
      c2 v0 = s[j], v1 = s[j + NR], v2 = s[j + 2 * NR], v3 = s[j + 3 * NR];
      v1 = cmul(v1, twid<LOG2N, INV>(qt, k * step));
      v2 = cmul(v2, twid<LOG2N, INV>(qt, 2 * k * step));
      v3 = cmul(v3, twid<LOG2N, INV>(qt, 3 * k * step));
      dft4<INV>(v0, v1, v2, v3);
      const int base = (j - k) * 4 + k;
      d[base] = v0;
      d[base + Ns] = v1;
      d[base + 2 * Ns] = v2;
      d[base + 3 * Ns] = v3;
    } else {
      c2 v0 = s[j], v1 = s[j + NR];
      v1 = cmul(v1, twid<LOG2N, INV>(qt, k * step));
      const int base = (j - k) * 2 + k;
      d[base] = v0 + v1;
      d[base + Ns] = v0 - v1;
    }
  }
}

// Full FFT of `frames` transforms starting in buf[0]; returns the buffer index holding the result.
template <int LOG2N, bool INV>
__device__ int fft(c2* buf0, c2* buf1, int frames, const c2* qt) {
  c2* b[2] = {buf0, buf1};
  int cur = 0, Ns = 1;
#pragma unroll
  for (int s = 0; s < LOG2N / 2; ++s) {
    stage<LOG2N, 4, INV>(b[cur], b[cur ^ 1], Ns, frames, qt);
    __syncthreads();
    cur ^= 1;
    Ns *= 4;
  }
  if constexpr (LOG2N & 1) {
    stage<LOG2N, 2, INV>(b[cur], b[cur ^ 1], Ns, frames, qt);
    __syncthreads();
    cur ^= 1;
  }
  return cur;
}

__device__ __forceinline__ int reflect(int i, int L) {
  i = i < 0 ? -i : i;
  return i >= L ? 2 * (L - 1) - i : i;
}


template <int LOG2N>
__global__ __launch_bounds__(NT) void mss_scale_kernel(const MssArgs a) {
  constexpr int N = 1 << LOG2N, H = N / 4, HALF = N / 2;
  constexpr int CF = CAP / N;                // frames per chunk
  constexpr int OWNF = RWIN / H;             // frames starting in the owned range
  __shared__ c2 bufs[2][CAP];
  __shared__ c2 qt[N / 4];
  __shared__ float acc[RWIN];
  __shared__ float red[2][NT / 64];

  const int w = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int L = (int)a.L;
  const float* p = a.pred + (long long)b * a.L;
  const float* q = a.target + (long long)b * a.L;
  const bool grad = a.dpred != nullptr;

  for (int r = tid; r < N / 4; r += NT) {
    double s, c;
    sincospi(2.0 * r / N, &s, &c);
    qt[r] = mk((float)c, (float)-s);
  }
  for (int i = tid; i < RWIN; i += NT) acc[i] = 0.f;
  __syncthreads();

  const int own_lo = w * RWIN;               // padded coordinates
  const int f_own0 = w * OWNF, f_own1 = min(f_own0 + OWNF, a.T);
  const int f_lo = grad ? max(f_own0 - 3, 0) : f_own0;
  float s_abs = 0.f, s_log = 0.f;

  for (int t0 = f_lo; t0 < f_own1; t0 += CF) {
    const int nf = min(CF, f_own1 - t0);
    // ---- load + window: z = w (p + i q)
    for (int e = tid; e < CF * N; e += NT) {
      const int fi = e / N, j = e - fi * N;
      c2 z = mk(0.f, 0.f);
      if (fi < nf) {
        const int src = reflect((t0 + fi) * H + j - HALF, L);
        const float wj = 0.5f - 0.5f * twid<LOG2N, false>(qt, j).x;  // periodic Hann
        z = mk(wj * p[src], wj * q[src]);
      }
      bufs[0][e] = z;
    }
    __syncthreads();
    const int fb = fft<LOG2N, false>(bufs[0], bufs[1], CF, qt);
    const c2* F = bufs[fb];
    c2* C = bufs[fb ^ 1];
    // ---- spectra, loss, gradient spectra packed in frame pairs
    constexpr int NPAIR = CF >= 2 ? CF / 2 : 1;
    for (int e = tid; e < NPAIR * (HALF + 1); e += NT) {
      const int m = e / (HALF + 1), f = e - m * (HALF + 1);
      c2 zg[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const int fi = CF >= 2 ? 2 * m + x : x;
        zg[x] = mk(0.f, 0.f);
        if ((CF >= 2 || x == 0) && fi < nf) {
          const c2 zf = F[fi * N + f], zr = F[fi * N + ((N - f) & (N - 1))];
          const c2 P = (zf + conjc(zr)) * 0.5f;
          const c2 D = zf - conjc(zr);
          const c2 Q = mk(D.y * 0.5f, -D.x * 0.5f);
          const float sp = sqrtf(P.x * P.x + P.y * P.y), st = sqrtf(Q.x * Q.x + Q.y * Q.y);
          const int t = t0 + fi;
          const float lp = logf(sp + a.eps), lt = logf(st + a.eps);
          if (t >= f_own0) {
            s_abs += fabsf(sp - st);
            s_log += fabsf(lp - lt);
          }
          if (grad && sp > 0.f) {
            const float sg = sp > st ? 1.f : (sp < st ? -1.f : 0.f);
            const float g = sg * (1.f + a.alpha / (sp + a.eps)) * a.inv_cnt;
            zg[x] = P * (g / sp);
          }
        }
      }
      if (grad) {
        c2* c = C + m * N;
        if (f == 0 || f == HALF) {
          c[f] = mk(zg[0].x, zg[1].x);
        } else {
          // H^a_f = Za/2, H^a_{n-f} = conj(Za)/2 (same for b); C = H^a + i H^b
          c[f] = mk(0.5f * (zg[0].x - zg[1].y), 0.5f * (zg[0].y + zg[1].x));
          c[N - f] = mk(0.5f * (zg[0].x + zg[1].y), 0.5f * (-zg[0].y + zg[1].x));
        }
      }
    }
    if (!grad) {
      __syncthreads();
      continue;
    }
    __syncthreads();
    c2* i0 = bufs[fb ^ 1];
    c2* i1 = bufs[fb];
    const int ib = fft<LOG2N, true>(i0, i1, NPAIR, qt);
    const c2* G = ib == 0 ? i0 : i1;
    // ---- windowed overlap-add into the owned range (each sample by one thread, frames in order)
    const int span_lo = max(own_lo, t0 * H), span_hi = min(own_lo + RWIN, (t0 + nf - 1) * H + N);
    for (int pp = span_lo + tid; pp < span_hi; pp += NT) {
      float v = acc[pp - own_lo];
      const int rel = pp - t0 * H;
      int fi0 = rel - N + 1 > 0 ? (rel - N + 1 + H - 1) / H : 0;
      int fi1 = min(nf - 1, rel / H);
      for (int fi = fi0; fi <= fi1; ++fi) {
        const int j = rel - fi * H;
        const float wj = 0.5f - 0.5f * twid<LOG2N, false>(qt, j).x;
        const c2 g = CF >= 2 ? G[(fi >> 1) * N + j] : G[j];
        v += wj * ((CF >= 2 && (fi & 1)) ? g.y : g.x);
      }
      acc[pp - own_lo] = v;
    }
    __syncthreads();
  }

  // ---- loss partials
  s_abs = wave_sum(s_abs);
  s_log = wave_sum(s_log);
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = s_abs;
    red[1][tid >> 6] = s_log;
  }
  __syncthreads();
  if (tid == 0) {
    float sa = 0.f, sl = 0.f;
    for (int i = 0; i < NT / 64; ++i) {
      sa += red[0][i];
      sl += red[1][i];
    }
    a.partial[((long long)b * a.nwg + w) * 2] = sa;
    a.partial[((long long)b * a.nwg + w) * 2 + 1] = sl;
  }
  if (!grad) return;
  // ---- gradient out: interior samples straight to dpred, reflect-pad samples to `edges`
  float* dp = a.dpred + (long long)b * a.L;
  float* ed = a.edges + (long long)b * N;
  const int own_hi = min(own_lo + RWIN, L + N);
  for (int pp = own_lo + tid; pp < own_hi; pp += NT) {
    const float v = acc[pp - own_lo];
    const int i = pp - HALF;
    if (i < 0) ed[pp] = v;
    else if (i >= L) ed[HALF + (i - L)] = v;
    else dp[i] = a.accumulate ? dp[i] + v : v;
  }
}

// Wave-local variant (the default): the same ownership (RWIN padded samples per workgroup, 3
// halo frames) and the same arithmetic, but every transform runs inside one wave, in place in
// that wave's LDS buffer (a radix-4 stage reads all its inputs into registers, then writes), so
// no workgroup barrier sits inside an FFT. Per round each wave takes 2 FB consecutive frames:
// pass A transforms the FB even ones and keeps their gradient spectra in registers, pass B the
// FB odd ones; the pair-packed Hermitian spectra C = H^a + i H^b then go through one inverse
// transform per pair. After a workgroup barrier every thread adds the round's frames covering
// its RWIN / 256 owned samples (kept in registers) in increasing frame order, so the summation
// order per sample is the frame order, as in the cooperative kernel above.
template <bool INV>
__device__ __forceinline__ c2 twq(const c2* qt, int m, int N) {  // W_N^m from the quarter table
  m &= N - 1;
  const int Q = N >> 2, q = m / Q, r = m & (Q - 1);
  const c2 w = qt[r];
  c2 o;
  if (q == 0) o = w;
  else if (q == 1) o = mk(w.y, -w.x);
  else if (q == 2) o = mk(-w.x, -w.y);
  else o = mk(-w.y, w.x);
  if (INV) o.y = -o.y;
  return o;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// FB = BW / N transforms of size N = 2^LOG2N, in place in s[0 .. BW) (Stockham order per stage:
// inputs read to registers, then outputs written), natural-order result.
template <int LOG2N, int BW, bool INV>
__device__ __forceinline__ void wave_fft(c2* s, const c2* qt, int lane) {
  constexpr int N = 1 << LOG2N, NR = N / 4, IT = BW / 4 / 64;
  int Ns = 1;
#pragma unroll
  for (int st = 0; st < LOG2N / 2; ++st) {
    c2 v[IT][4];
    int ln = lane;
    __asm__ volatile("" : "+v"(ln));  // lane-derived addresses formed per stage, not kept live
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int idx = ln + 64 * it, fr = idx / NR, j = idx - fr * NR;
      const c2* src = s + fr * N + j;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[it][r] = src[r * NR];
    }
    wave_sync();
    const int step = N / (Ns * 4);
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int idx = ln + 64 * it, fr = idx / NR, j = idx - fr * NR;
      const int k = j & (Ns - 1);
      if (st > 0) {  // k step < N / 4: one quarter-table entry, its square and cube
        c2 w1 = qt[k * step];
        if (INV) w1.y = -w1.y;
        const c2 w2 = cmul(w1, w1);
        v[it][1] = cmul(v[it][1], w1);
        v[it][2] = cmul(v[it][2], w2);
        v[it][3] = cmul(v[it][3], cmul(w2, w1));
      }
      dft4<INV>(v[it][0], v[it][1], v[it][2], v[it][3]);
      c2* d = s + fr * N + (j - k) * 4 + k;
#pragma unroll
      for (int r = 0; r < 4; ++r) d[r * Ns] = v[it][r];
    }
    wave_sync();
    Ns *= 4;
  }
  if constexpr (LOG2N & 1) {
    constexpr int NR2 = N / 2, IT2 = BW / 2 / 64;
    c2 v[IT2][2];
    int ln = lane;
    __asm__ volatile("" : "+v"(ln));
#pragma unroll
    for (int it = 0; it < IT2; ++it) {
      const int idx = ln + 64 * it, fr = idx / NR2, j = idx - fr * NR2;
      v[it][0] = s[fr * N + j];
      v[it][1] = s[fr * N + j + NR2];
    }
    wave_sync();
#pragma unroll
    for (int it = 0; it < IT2; ++it) {
      const int idx = ln + 64 * it, fr = idx / NR2, j = idx - fr * NR2;
      const int k = j & (Ns - 1);
      const c2 b = cmul(v[it][1], twq<INV>(qt, k, 2 * Ns));
      c2* d = s + fr * N + (j - k) * 2 + k;
      d[0] = v[it][0] + b;
      d[Ns] = v[it][0] - b;
    }
    wave_sync();
  }
}

template <int LOG2N>
__global__ __launch_bounds__(256, LOG2N == 11 ? 2 : 4) void mss_wave_kernel(const MssArgs a) {
  constexpr int N = 1 << LOG2N, H = N / 4, HALF = N / 2, NBIN = HALF + 1;
  constexpr int W = 4;                       // waves per workgroup
  constexpr int BW = N > 1024 ? N : 1024;    // complex per wave buffer
  constexpr int FB = BW / N;                 // transforms per pass
  constexpr int GF = 2 * FB;                 // frames per wave per round
  constexpr int RF = W * GF;                 // frames per round
  constexpr int NE = (FB * NBIN + 63) / 64;  // spectrum entries per lane
  constexpr int OWN = RWIN / 256;            // owned samples per thread
  __shared__ __attribute__((aligned(16))) c2 buf[W * BW];
  __shared__ c2 qt[N / 4];
  __shared__ float hw[N];
  __shared__ float red[2][W];

  const int w = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int L = (int)a.L;
  const float* p = a.pred + (long long)b * a.L;
  const float* q = a.target + (long long)b * a.L;
  const bool grad = a.dpred != nullptr;
  for (int r = tid; r < N / 4; r += 256) {
    double sn, cs;
    sincospi(2.0 * r / N, &sn, &cs);
    qt[r] = mk((float)cs, (float)-sn);
  }
  for (int j = tid; j < N; j += 256) {
    double sn, cs;
    sincospi(2.0 * j / N, &sn, &cs);
    hw[j] = (float)(0.5 - 0.5 * cs);  // periodic Hann
  }
  __syncthreads();

  const int own_lo = w * RWIN;
  const int f_own0 = w * (RWIN / H), f_own1 = min(f_own0 + RWIN / H, a.T);
  const int f_lo = grad ? max(f_own0 - 3, 0) : f_own0;
  c2* S = buf + wave * BW;
  float acc[OWN];
#pragma unroll
  for (int i = 0; i < OWN; ++i) acc[i] = 0.f;
  float s_abs = 0.f, s_log = 0.f;

#pragma unroll 1
  for (int t_round = f_lo; t_round < f_own1; t_round += RF) {
    const int t_base = t_round + wave * GF;  // this wave's first frame
    if (t_base < f_own1) {                   // wave-uniform
      c2 zga[NE], zgb[NE];
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
        // load + window FB frames t_base + 2m + pass: z = w (p + i q)
#pragma unroll 4
        for (int k = 0; k < BW / 64; ++k) {
          const int e = lane + 64 * k, m = e / N, j = e - m * N;
          const int t = t_base + 2 * m + pass;
          c2 z = mk(0.f, 0.f);
          if (t < f_own1) {
            const int src = reflect(t * H + j - HALF, L);
            z = mk(hw[j] * p[src], hw[j] * q[src]);
          }
          S[e] = z;
        }
        wave_sync();
        wave_fft<LOG2N, BW, false>(S, qt, lane);
        // spectra, loss, gradient spectra (registers)
#pragma unroll
        for (int jj = 0; jj < NE; ++jj) {
          int ln = lane;
          __asm__ volatile("" : "+v"(ln));  // per-entry indices, not kept live across the loop
          const int e = ln + 64 * jj, m = e / NBIN, f = e - m * NBIN;
          const int t = t_base + 2 * m + pass;
          c2 zg = mk(0.f, 0.f);
          if (e < FB * NBIN && t < f_own1) {
            const c2 zf = S[m * N + f], zr = S[m * N + ((N - f) & (N - 1))];
            const c2 P = (zf + conjc(zr)) * 0.5f;
            const c2 D = zf - conjc(zr);
            const c2 Q = mk(D.y * 0.5f, -D.x * 0.5f);
            // hardware sqrt / log2 / rcp (1 ulp): the library forms add ~10 instructions each
            const float sp = __builtin_amdgcn_sqrtf(P.x * P.x + P.y * P.y);
            const float st = __builtin_amdgcn_sqrtf(Q.x * Q.x + Q.y * Q.y);
            const float lp = __log2f(sp + a.eps) * 0.69314718055994531f;
            const float lt = __log2f(st + a.eps) * 0.69314718055994531f;
            if (t >= f_own0) {
              s_abs += fabsf(sp - st);
              s_log += fabsf(lp - lt);
            }
            if (grad && sp > 0.f) {
              const float sg = sp > st ? 1.f : (sp < st ? -1.f : 0.f);
              const float g = sg * (1.f + a.alpha / (sp + a.eps)) * a.inv_cnt;
              zg = P * (g * __builtin_amdgcn_rcpf(sp));
            }
          }
          if (pass == 0) zga[jj] = zg;
          else zgb[jj] = zg;
        }
        wave_sync();  // every lane has read the spectra before S is overwritten
      }
      if (grad) {
        // C = H^a + i H^b per pair (H^a_f = Za/2, H^a_{n-f} = conj(Za)/2)
#pragma unroll
        for (int jj = 0; jj < NE; ++jj) {
          int ln = lane;
          __asm__ volatile("" : "+v"(ln));
          const int e = ln + 64 * jj, m = e / NBIN, f = e - m * NBIN;
          if (e < FB * NBIN) {
            const c2 za = zga[jj], zb = zgb[jj];
            c2* c = S + m * N;
            if (f == 0 || f == HALF) {
              c[f] = mk(za.x, zb.x);
            } else {
              c[f] = mk(0.5f * (za.x - zb.y), 0.5f * (za.y + zb.x));
              c[N - f] = mk(0.5f * (za.x + zb.y), 0.5f * (-za.y + zb.x));
            }
          }
        }
        wave_sync();
        wave_fft<LOG2N, BW, true>(S, qt, lane);
      }
    }
    if (!grad) continue;  // uniform over the workgroup: no barrier needed
    __syncthreads();      // every wave's gradient frames are in its buffer
    // windowed overlap-add of the round's frames into the owned samples, frames in order
    const int r_hi = min(t_round + RF, f_own1);
#pragma unroll
    for (int i = 0; i < OWN; ++i) {
      const int sp = own_lo + tid + 256 * i;  // padded coordinate
      const int th = sp / H;
      const int t0 = max(max(th - 3, t_round), 0), t1 = min(th, r_hi - 1);
      float v = acc[i];
      for (int t = t0; t <= t1; ++t) {
        const int j = sp - t * H;
        const int rel = t - t_round, ww = rel / GF, m = (rel - ww * GF) >> 1;
        const c2 g = buf[ww * BW + m * N + j];
        v += hw[j] * ((rel & 1) ? g.y : g.x);
      }
      acc[i] = v;
    }
    __syncthreads();  // the buffers are read before the next round overwrites them
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
  float* dp = a.dpred + (long long)b * a.L;
  float* ed = a.edges + (long long)b * N;
  const int own_hi = min(own_lo + RWIN, L + N);
#pragma unroll
  for (int i = 0; i < OWN; ++i) {
    const int pp = own_lo + tid + 256 * i;
    if (pp >= own_hi) continue;
    const float v = acc[i];
    const int x = pp - HALF;
    if (x < 0) ed[pp] = v;
    else if (x >= L) ed[HALF + (x - L)] = v;
    else dp[x] = a.accumulate ? dp[x] + v : v;
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
};

__global__ void mss_fold_kernel(const FoldArgs a) {
  const int b = blockIdx.x;
  const int L = (int)a.L;
  float* dp = a.dpred + (long long)b * a.L;
  for (int s = 0; s < a.nsz; ++s) {
    const int n = a.n[s], half = n / 2;
    const float* ed = a.edges + a.off[s] + (long long)b * n;
    // head: padded p < n/2 is x[n/2 - p]; tail: x[2(L-1) - (L + k)] = x[L - 2 - k]
    for (int k = threadIdx.x; k < half; k += blockDim.x) {
      dp[half - k] += ed[k];
    }
    __syncthreads();
    for (int k = threadIdx.x; k < half; k += blockDim.x) {
      dp[L - 2 - k] += ed[half + k];
    }
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

__global__ void mss_loss_kernel(const LossArgs a) {
  __shared__ double red[4];
  double tot = 0.0;
  for (int s = 0; s < a.nsz; ++s) {
    double sa = 0.0, sl = 0.0;
    for (int i = threadIdx.x; i < a.cnt[s]; i += blockDim.x) {
      sa += a.partial[a.off[s] + 2 * i];
      sl += a.partial[a.off[s] + 2 * i + 1];
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

// MST_MSS_LEGACY=1: the workgroup-cooperative kernel (A/B)
bool mss_legacy() {
  static const bool v = [] {
    const char* e = getenv("MST_MSS_LEGACY");
    return e && atoi(e) != 0;
  }();
  return v;
}

// MST_MSS_REG=0: n = 1024 on mss_wave_kernel instead of the register-resident FFT (A/B)
bool mss_reg() {
  static const bool v = [] {
    const char* e = getenv("MST_MSS_REG");
    return !(e && e[0] == '0');
  }();
  return v;
}

int log2i(int n) {
  int l = 0;
  while ((1 << l) < n) ++l;
  return (1 << l) == n ? l : -1;
}

struct Plan {
  int nsz;
  int n[8], T[8], nwg[8];
  long long part_off[8], edge_off[8];
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
  pl.bytes = (size_t)(part + edge) * sizeof(float);
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
  for (int s = 0; s < pl.nsz; ++s) {
    MssArgs a;
    a.pred = pred;
    a.target = target;
    a.L = L;
    a.T = pl.T[s];
    a.nwg = pl.nwg[s];
    a.alpha = alpha;
    a.eps = eps;
    a.inv_cnt = (float)(1.0 / ((double)B * pl.T[s] * (pl.n[s] / 2 + 1)));
    a.dpred = dpred;
    a.accumulate = s > 0;
    a.edges = w + pl.edge_off[s];
    a.partial = w + pl.part_off[s];
    dim3 grid(pl.nwg[s], (unsigned)B);
    if (mss_legacy()) {
      switch (log2i(pl.n[s])) {
        case 6: mss_scale_kernel<6><<<grid, NT, 0, st>>>(a); break;
        case 7: mss_scale_kernel<7><<<grid, NT, 0, st>>>(a); break;
        case 8: mss_scale_kernel<8><<<grid, NT, 0, st>>>(a); break;
        case 9: mss_scale_kernel<9><<<grid, NT, 0, st>>>(a); break;
        case 10: mss_scale_kernel<10><<<grid, NT, 0, st>>>(a); break;
        default: mss_scale_kernel<11><<<grid, NT, 0, st>>>(a); break;
      }
    } else {
      switch (log2i(pl.n[s])) {
        case 6: mss_wave_kernel<6><<<grid, 256, 0, st>>>(a); break;
        case 7: mss_wave_kernel<7><<<grid, 256, 0, st>>>(a); break;
        case 8: mss_wave_kernel<8><<<grid, 256, 0, st>>>(a); break;
        case 9: mss_wave_kernel<9><<<grid, 256, 0, st>>>(a); break;
        case 10:
          if (mss_reg()) mss_fft1024_launch(a, grid.x, grid.y, st);
          else mss_wave_kernel<10><<<grid, 256, 0, st>>>(a);
          break;
        default:
          if (mss_reg()) mss_fft2048_launch(a, grid.x, grid.y, st);
          else mss_wave_kernel<11><<<grid, 256, 0, st>>>(a);
          break;
      }
    }
    MST_CHECK_LAUNCH();
  }
  if (dpred) {
    FoldArgs f;
    f.dpred = dpred;
    f.edges = w;
    f.L = L;
    f.B = (int)B;
    f.nsz = pl.nsz;
    for (int s = 0; s < pl.nsz; ++s) {
      f.n[s] = pl.n[s];
      f.off[s] = pl.edge_off[s];
    }
    mss_fold_kernel<<<(unsigned)B, 256, 0, st>>>(f);
    MST_CHECK_LAUNCH();
  }
  LossArgs la;
  la.partial = w;
  la.nsz = pl.nsz;
  la.alpha = alpha;
  la.loss = loss;
  for (int s = 0; s < pl.nsz; ++s) {
    la.off[s] = pl.part_off[s];
    la.cnt[s] = (int)(B * pl.nwg[s]);
    la.inv_cnt[s] = (float)(1.0 / ((double)B * pl.T[s] * (pl.n[s] / 2 + 1)));
  }
  mss_loss_kernel<<<1, 256, 0, st>>>(la);
  MST_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
