// Microbenchmark (dev tool): a bf16x6 NT GEMM on PRE-SPLIT operand planes, C[m][n] = sum_k
// A[m][k] B[n][k] with A = A0 + A1 + A2 and B = B0 + B1 + B2 held as three bf16 planes each in HBM
// ([rows][K], K contiguous). The tiles go straight into LDS by buffer_load ... lds (no VGPRs, no
// split VALU), in the 128 x 256 kernel's swizzled plane layout (gemm.hip), so the main loop is
// ds_read + MFMA only. Question it answers: what TF/s (fp32 products) a pre-split operand path
// reaches on the training step's GEMM shapes, against the register-split kernels' 130-165.
//
// build: make -C tools/micro gemm_planes ; run: tools/micro/gemm_planes
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr int BM = 128, BN = 256, BK = 32, NT = 512;
constexpr int PA = BM * BK, PB = BN * BK;           // bf16 elements per A / B plane tile
constexpr int STAGE = 3 * PA + 3 * PB;              // 72 KB of bf16 per stage
constexpr int LDS_BYTES = 2 * STAGE * 2;            // two stages: 144 KB

__device__ __forceinline__ int pl_swz(int row) {
  return ((row >> 2) & 1) | (((row >> 1) ^ (row >> 3)) & 1) << 1;
}
__device__ __forceinline__ int pl_off(int row, int q) { return row * BK + 8 * (q ^ pl_swz(row)); }

struct Split3 {
  bf16x8 h, m, l;
};
template <int PS>
__device__ __forceinline__ Split3 ld_planes(const __bf16* base, int row, int q) {
  const __bf16* p = base + pl_off(row, q);
  Split3 s;
  s.h = *reinterpret_cast<const bf16x8*>(p);
  s.m = *reinterpret_cast<const bf16x8*>(p + PS);
  s.l = *reinterpret_cast<const bf16x8*>(p + 2 * PS);
  return s;
}
__device__ __forceinline__ f32x16 mfma_x6(const Split3& a, const Split3& b, f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.l, b.h, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.l, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.m, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.h, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.m, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.h, acc, 0, 0, 0);
  return acc;
}

struct PP {
  const __bf16* A;  // 3 planes, plane stride sa elements, row stride lda
  const __bf16* B;
  long long sa, sb;
  int M, N, K, lda, ldb;
  float* C;
  int ldc;
};

__device__ __forceinline__ int xcd_order(int w, int W) {
  const int q = W >> 3, r = W & 7, xcd = w & 7;
  return xcd * q + min(xcd, r) + (w >> 3);
}


// LDS-DMA as inline asm: hipcc does not model it, so it does not insert the s_waitcnt vmcnt(0) it
// puts before every ds_read that may alias a builtin LDS-DMA (which waits for the NEXT stage's
// pieces before reading the current one, i.e. exposes the DMA latency on every K tile). M0 is
// written and restored inside the statement; the kernel counts vmcnt itself.
__device__ __forceinline__ void dma_asm(rsrc_t rs, unsigned lds_addr, uint32_t voff, int soff) {
  unsigned keep;
  asm volatile(
      "s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rs), "s"(lds_addr), "s"(soff)
      : "memory");
}
template <int ASM>
__device__ __forceinline__ void dma16(rsrc_t rs, char* lds, int byte_off, uint32_t voff, int soff) {
  if constexpr (ASM) {
    dma_asm(rs, __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds + byte_off), voff, soff);
  } else {
    auto* dst = (__attribute__((address_space(3))) void*)(lds + byte_off);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, dst, 16, voff, soff, 0, 0);
  }
}

// MODE 0: builtin DMA (v1); 1: asm DMA (v5); 2: asm DMA spread over the MFMAs (v6)
__device__ unsigned long long g_clk[4 * 65536];  // MODE 3: per workgroup memtime / realtime at start / end

template <int MODE>
__global__ __launch_bounds__(NT, 1) void gemm_planes_kernel(const PP p) {
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  const unsigned wg_lin = blockIdx.x + gridDim.x * blockIdx.y;
  if (MODE == 3 && threadIdx.x == 0 && wg_lin < 65536) {
    g_clk[4 * wg_lin] = __builtin_amdgcn_s_memtime();
    g_clk[4 * wg_lin + 1] = __builtin_amdgcn_s_memrealtime();
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nx = (p.N + BN - 1) / BN, ny = (p.M + BM - 1) / BM;
  const int t = xcd_order(blockIdx.x + nx * blockIdx.y, nx * ny);
  // runs of 8 M tiles x all N tiles (gemm.hip tile_of)
  const int GM = ny < 8 ? ny : 8, grp = t / (GM * nx), fm = grp * GM;
  const int gm = ny - fm < GM ? ny - fm : GM, tg = t - grp * GM * nx;
  const int m0 = (fm + tg % gm) * BM, n0 = (tg / gm) * BN;
  // operand descriptors: rows past M / N read zeros (bounded buffer loads)
  const rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0,
                                                      (int)((2 * p.sa + (long long)p.M * p.lda) * 2), 0x00020000);
  const rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0,
                                                      (int)((2 * p.sb + (long long)p.N * p.ldb) * 2), 0x00020000);
  // this wave's 9 glds instructions per stage: j = wave + 8 i; j < 24 are A (plane j / 8, rows
  // 16 (j % 8) ..), the rest B (plane (j - 24) / 16, rows 16 ((j - 24) % 16) ..). Lane l fills
  // LDS bytes 16 l of the instruction's 1 KB: row r0 + l / 4, slot l % 4 = quad q ^ swz(row).
  uint32_t voff[9];
  int isA[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int j = wave + 8 * i;
    const bool a = j < 24;
    const int jj = a ? j : j - 24;
    const int plane = a ? jj / 8 : jj / 16;
    const int r = (a ? jj % 8 : jj % 16) * 16 + (lane >> 2);
    const int q = (lane & 3) ^ pl_swz(r);
    const long long row = a ? (long long)(m0 + r) : (long long)(n0 + r);
    const bool in = a ? (m0 + r < p.M) : (n0 + r < p.N);
    const long long e = plane * (a ? p.sa : p.sb) + row * (a ? p.lda : p.ldb) + 8 * q;
    voff[i] = in ? (uint32_t)(e * 2) : 0x7FFFFFF0u;
    isA[i] = a;
  }
  auto piece = [&](int i, int stage, int kt) __attribute__((always_inline)) {
    const int j = wave + 8 * i;
    if (j < 24) dma16<MODE != 0>(rA, lds, stage * STAGE * 2 + j * 1024, voff[i], kt * BK * 2);
    else dma16<MODE != 0>(rB, lds, stage * STAGE * 2 + j * 1024, voff[i], kt * BK * 2);
  };
  auto issue = [&](int stage, int kt) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 9; ++i) piece(i, stage, kt);
  };
  const int g = __builtin_amdgcn_readfirstlane(tid >> 8);
  const int wm = (wave >> 1) & 1, wn = wave & 1;
  const int r32 = lane & 31, h = lane >> 5;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = (p.K + BK - 1) / BK;
  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 1;
    const bool more = kt + 1 < nk;
    if (MODE != 2 && more) issue(st ^ 1, kt + 1);  // MODE 3: as MODE 1
    const __bf16* Ap = reinterpret_cast<const __bf16*>(lds) + st * STAGE;
    const __bf16* Bp = Ap + 3 * PA;
    const int ra0 = wm * 64 + r32, rb0 = 128 * g + wn * 64 + r32;
    // MODE 2: the next stage's 9 pieces in four groups after the reads of each 12-MFMA group
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const Split3 b0 = ld_planes<PB>(Bp, rb0, 2 * s + h), b1 = ld_planes<PB>(Bp, rb0 + 32, 2 * s + h);
      const Split3 a0 = ld_planes<PA>(Ap, ra0, 2 * s + h);
      if (MODE == 2 && more) {  // pieces 0, 1 (s = 0) / 5, 6 (s = 1)
        piece(5 * s, st ^ 1, kt + 1);
        piece(5 * s + 1, st ^ 1, kt + 1);
      }
      acc[0][0] = mfma_x6(a0, b0, acc[0][0]);
      acc[0][1] = mfma_x6(a0, b1, acc[0][1]);
      const Split3 a1 = ld_planes<PA>(Ap, ra0 + 32, 2 * s + h);
      if (MODE == 2 && more) {  // pieces 2, 3, 4 (s = 0) / 7, 8 (s = 1)
        piece(5 * s + 2, st ^ 1, kt + 1);
        piece(5 * s + 3, st ^ 1, kt + 1);
        if (s == 0) piece(4, st ^ 1, kt + 1);
      }
      acc[1][0] = mfma_x6(a1, b0, acc[1][0]);
      acc[1][1] = mfma_x6(a1, b1, acc[1][1]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // epilogue through LDS (128 x 256 floats aliases the stages)
  float* Cs = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ml = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int nl = 128 * g + wn * 64 + j * 32 + r32;
        Cs[ml * BN + nl] = acc[i][j][r];
      }
  __syncthreads();
  const int nl = tid & (BN - 1);
  if (n0 + nl < p.N)
    for (int ml = tid >> 8; ml < BM && m0 + ml < p.M; ml += 2) p.C[(long long)(m0 + ml) * p.ldc + n0 + nl] = Cs[ml * BN + nl];
  if (MODE == 3 && threadIdx.x == 0 && wg_lin < 65536) {
    g_clk[4 * wg_lin + 2] = __builtin_amdgcn_s_memtime();
    g_clk[4 * wg_lin + 3] = __builtin_amdgcn_s_memrealtime();
  }
}


// ---- variants 8-12: v5 (asm DMA) plus: CLK in-kernel clock stamps (s_memtime / s_memrealtime per
// workgroup); STAG a stagger (MI355X_MICROARCH.md "two waves per SIMD" item 9): waves 4-7 (the
// second wave on each SIMD) run each K tile's second 16-deep half one barrier late, from fragments
// read into registers before the barrier, so after every barrier one wave per SIMD issues MFMAs
// at once while its partner reads its next fragments; PRIO s_setprio 1 for waves 4-7 (item 4).
template <bool CLK, bool STAG, bool PRIO>
__global__ __launch_bounds__(NT, 1) void gemm_planes_x_kernel(const PP p) {
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  const unsigned wg_lin = blockIdx.x + gridDim.x * blockIdx.y;
  if (CLK && threadIdx.x == 0 && wg_lin < 65536) {
    g_clk[4 * wg_lin] = __builtin_amdgcn_s_memtime();
    g_clk[4 * wg_lin + 1] = __builtin_amdgcn_s_memrealtime();
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nx = (p.N + BN - 1) / BN, ny = (p.M + BM - 1) / BM;
  const int t = xcd_order(blockIdx.x + nx * blockIdx.y, nx * ny);
  const int GM = ny < 8 ? ny : 8, grp = t / (GM * nx), fm = grp * GM;
  const int gm = ny - fm < GM ? ny - fm : GM, tg = t - grp * GM * nx;
  const int m0 = (fm + tg % gm) * BM, n0 = (tg / gm) * BN;
  const rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0,
                                                      (int)((2 * p.sa + (long long)p.M * p.lda) * 2), 0x00020000);
  const rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0,
                                                      (int)((2 * p.sb + (long long)p.N * p.ldb) * 2), 0x00020000);
  uint32_t voff[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int j = wave + 8 * i;
    const bool a = j < 24;
    const int jj = a ? j : j - 24;
    const int plane = a ? jj / 8 : jj / 16;
    const int r = (a ? jj % 8 : jj % 16) * 16 + (lane >> 2);
    const int q = (lane & 3) ^ pl_swz(r);
    const long long row = a ? (long long)(m0 + r) : (long long)(n0 + r);
    const bool in = a ? (m0 + r < p.M) : (n0 + r < p.N);
    const long long e = plane * (a ? p.sa : p.sb) + row * (a ? p.lda : p.ldb) + 8 * q;
    voff[i] = in ? (uint32_t)(e * 2) : 0x7FFFFFF0u;
  }
  auto issue = [&](int stage, int kt) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int j = wave + 8 * i;
      if (j < 24) dma16<1>(rA, lds, stage * STAGE * 2 + j * 1024, voff[i], kt * BK * 2);
      else dma16<1>(rB, lds, stage * STAGE * 2 + j * 1024, voff[i], kt * BK * 2);
    }
  };
  const int g = __builtin_amdgcn_readfirstlane(tid >> 8);
  const int wm = (wave >> 1) & 1, wn = wave & 1;
  const int r32 = lane & 31, h = lane >> 5;
  const int ra0 = wm * 64 + r32, rb0 = 128 * g + wn * 64 + r32;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  auto half = [&](const Split3& a0, const Split3& a1, const Split3& b0, const Split3& b1)
      __attribute__((always_inline)) {
    acc[0][0] = mfma_x6(a0, b0, acc[0][0]);
    acc[0][1] = mfma_x6(a0, b1, acc[0][1]);
    acc[1][0] = mfma_x6(a1, b0, acc[1][0]);
    acc[1][1] = mfma_x6(a1, b1, acc[1][1]);
  };
  const int nk = (p.K + BK - 1) / BK;
  if (PRIO && wave >= 4) __builtin_amdgcn_s_setprio(1);
  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const bool late = STAG && wave >= 4;  // wave-uniform
  if (!late) {
    for (int kt = 0; kt < nk; ++kt) {
      const int st = kt & 1;
      if (kt + 1 < nk) issue(st ^ 1, kt + 1);
      const __bf16* Ap = reinterpret_cast<const __bf16*>(lds) + st * STAGE;
      const __bf16* Bp = Ap + 3 * PA;
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
        const Split3 b0 = ld_planes<PB>(Bp, rb0, 2 * s + h), b1 = ld_planes<PB>(Bp, rb0 + 32, 2 * s + h);
        const Split3 a0 = ld_planes<PA>(Ap, ra0, 2 * s + h);
        acc[0][0] = mfma_x6(a0, b0, acc[0][0]);
        acc[0][1] = mfma_x6(a0, b1, acc[0][1]);
        const Split3 a1 = ld_planes<PA>(Ap, ra0 + 32, 2 * s + h);
        acc[1][0] = mfma_x6(a1, b0, acc[1][0]);
        acc[1][1] = mfma_x6(a1, b1, acc[1][1]);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    Split3 pa0, pa1, pb0, pb1;  // the previous tile's second half, read before the barrier
    for (int kt = 0; kt < nk; ++kt) {
      const int st = kt & 1;
      if (kt + 1 < nk) issue(st ^ 1, kt + 1);
      if (kt > 0) half(pa0, pa1, pb0, pb1);
      const __bf16* Ap = reinterpret_cast<const __bf16*>(lds) + st * STAGE;
      const __bf16* Bp = Ap + 3 * PA;
      {
        const Split3 b0 = ld_planes<PB>(Bp, rb0, h), b1 = ld_planes<PB>(Bp, rb0 + 32, h);
        const Split3 a0 = ld_planes<PA>(Ap, ra0, h), a1 = ld_planes<PA>(Ap, ra0 + 32, h);
        half(a0, a1, b0, b1);
      }
      pb0 = ld_planes<PB>(Bp, rb0, 2 + h);
      pb1 = ld_planes<PB>(Bp, rb0 + 32, 2 + h);
      pa0 = ld_planes<PA>(Ap, ra0, 2 + h);
      pa1 = ld_planes<PA>(Ap, ra0 + 32, 2 + h);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    if (nk > 0) half(pa0, pa1, pb0, pb1);
  }
  float* Cs = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ml = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int nl = 128 * g + wn * 64 + j * 32 + r32;
        Cs[ml * BN + nl] = acc[i][j][r];
      }
  __syncthreads();
  const int nl = tid & (BN - 1);
  if (n0 + nl < p.N)
    for (int ml = tid >> 8; ml < BM && m0 + ml < p.M; ml += 2) p.C[(long long)(m0 + ml) * p.ldc + n0 + nl] = Cs[ml * BN + nl];
  if (CLK && threadIdx.x == 0 && wg_lin < 65536) {
    g_clk[4 * wg_lin + 2] = __builtin_amdgcn_s_memtime();
    g_clk[4 * wg_lin + 3] = __builtin_amdgcn_s_memrealtime();
  }
}

// ---- variant 2: 256 x 256 tile, BK = 16, three LDS stages (48 KB each) with one stage of
// buffer_load ... lds in flight across each barrier (counted vmcnt, raw s_barrier). 8 waves as
// 2 (M) x 4 (N), wave tile 128 x 64 (4 x 2 blocks of 32 x 32). Plane rows are 32 B (two 16-byte
// quads), quad slot XOR (row >> 3) & 1: conflict-free for the ds_read_b128 fragment reads.
constexpr int B2M = 256, B2N = 256, B2K = 16;
constexpr int P2 = 256 * B2K;          // bf16 elements per plane tile
constexpr int STAGE2 = 6 * P2;         // A 3 planes + B 3 planes = 48 KB
constexpr int NST2 = 3;

__device__ __forceinline__ int off2(int row, int q) { return row * B2K + 8 * (q ^ ((row >> 3) & 1)); }
__device__ __forceinline__ Split3 ld2(const __bf16* base, int row, int q) {
  const __bf16* p = base + off2(row, q);
  Split3 s;
  s.h = *reinterpret_cast<const bf16x8*>(p);
  s.m = *reinterpret_cast<const bf16x8*>(p + P2);
  s.l = *reinterpret_cast<const bf16x8*>(p + 2 * P2);
  return s;
}

__global__ __launch_bounds__(NT, 1) void gemm_planes2_kernel(const PP p) {
  __shared__ __attribute__((aligned(16))) char lds[NST2 * STAGE2 * 2];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nx = (p.N + B2N - 1) / B2N, ny = (p.M + B2M - 1) / B2M;
  const int t = xcd_order(blockIdx.x + nx * blockIdx.y, nx * ny);
  const int GM = ny < 8 ? ny : 8, grp = t / (GM * nx), fm = grp * GM;
  const int gm = ny - fm < GM ? ny - fm : GM, tg = t - grp * GM * nx;
  const int m0 = (fm + tg % gm) * B2M, n0 = (tg / gm) * B2N;
  const rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0,
                                                      (int)((2 * p.sa + (long long)p.M * p.lda) * 2), 0x00020000);
  const rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0,
                                                      (int)((2 * p.sb + (long long)p.N * p.ldb) * 2), 0x00020000);
  // 48 one-KB pieces per stage, 6 per wave: j = wave + 8 i; j < 24 A (plane j / 8, rows
  // 32 (j % 8) ..), else B. Lane l: row r0 + l / 2, slot l % 2 = quad q ^ swz(row).
  uint32_t voff[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int j = wave + 8 * i;
    const bool a = j < 24;
    const int jj = a ? j : j - 24;
    const int plane = jj >> 3;
    const int r = (jj & 7) * 32 + (lane >> 1);
    const int q = (lane & 1) ^ ((r >> 3) & 1);
    const long long row = a ? (long long)(m0 + r) : (long long)(n0 + r);
    const bool in = a ? (m0 + r < p.M) : (n0 + r < p.N);
    const long long e = plane * (a ? p.sa : p.sb) + row * (a ? p.lda : p.ldb) + 8 * q;
    voff[i] = in ? (uint32_t)(e * 2) : 0x7FFFFFF0u;
  }
  auto issue = [&](int stage, int kt) __attribute__((always_inline)) {
    const int soff = kt * B2K * 2;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int j = wave + 8 * i;
      auto* dst = (__attribute__((address_space(3))) void*)(lds + stage * STAGE2 * 2 + j * 1024);
      if (j < 24) __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, dst, 16, voff[i], soff, 0, 0);
      else __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, dst, 16, voff[i], soff, 0, 0);
    }
  };
  const int wm = wave >> 2, wn = wave & 3;
  const int r32 = lane & 31, h = lane >> 5;
  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = (p.K + B2K - 1) / B2K;
  issue(0, 0);
  if (nk > 1) issue(1, 1);
  if (nk > 1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  int st = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 2 < nk) issue(st == 0 ? 2 : st - 1, kt + 2);  // the stage read one iteration ago
    const __bf16* Ap = reinterpret_cast<const __bf16*>(lds) + st * STAGE2;
    const __bf16* Bp = Ap + 3 * P2;
    const Split3 b0 = ld2(Bp, wn * 64 + r32, h), b1 = ld2(Bp, wn * 64 + 32 + r32, h);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const Split3 a = ld2(Ap, wm * 128 + 32 * i + r32, h);
      acc[i][0] = mfma_x6(a, b0, acc[i][0]);
      acc[i][1] = mfma_x6(a, b1, acc[i][1]);
    }
    // retire the next stage's DMA (this wave's part), keep the one after it in flight
    if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    st = st == 2 ? 0 : st + 1;
  }
  // epilogue straight from the accumulators (lane: column r32, rows in the registers)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + 32 * j + r32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 128 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < p.M && n < p.N) p.C[(long long)m * p.ldc + n] = acc[i][j][r];
      }
    }
}

// ---- variant 3: 128 x 128 tile, BK = 16, three 24 KB stages, 256 threads (2 x 2 waves of 64 x 64),
// TWO workgroups per CU: one workgroup's barrier bubble is filled by the other's MFMAs.
constexpr int P3 = 128 * B2K;   // bf16 elements per plane tile
constexpr int STAGE3 = 6 * P3;  // 24 KB
__device__ __forceinline__ Split3 ld3(const __bf16* base, int row, int q) {
  const __bf16* p = base + off2(row, q);
  Split3 s;
  s.h = *reinterpret_cast<const bf16x8*>(p);
  s.m = *reinterpret_cast<const bf16x8*>(p + P3);
  s.l = *reinterpret_cast<const bf16x8*>(p + 2 * P3);
  return s;
}

__global__ __launch_bounds__(256, 2) void gemm_planes3_kernel(const PP p) {
  __shared__ __attribute__((aligned(16))) char lds[3 * STAGE3 * 2];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nx = (p.N + 127) / 128, ny = (p.M + 127) / 128;
  const int t = xcd_order(blockIdx.x + nx * blockIdx.y, nx * ny);
  const int GM = ny < 8 ? ny : 8, grp = t / (GM * nx), fm = grp * GM;
  const int gm = ny - fm < GM ? ny - fm : GM, tg = t - grp * GM * nx;
  const int m0 = (fm + tg % gm) * 128, n0 = (tg / gm) * 128;
  const rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0,
                                                      (int)((2 * p.sa + (long long)p.M * p.lda) * 2), 0x00020000);
  const rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0,
                                                      (int)((2 * p.sb + (long long)p.N * p.ldb) * 2), 0x00020000);
  // 24 one-KB pieces per stage, 6 per wave: j = wave + 4 i; j < 12 A (plane j / 4, rows 32 (j % 4)), else B
  uint32_t voff[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int j = wave + 4 * i;
    const bool a = j < 12;
    const int jj = a ? j : j - 12;
    const int plane = jj >> 2;
    const int r = (jj & 3) * 32 + (lane >> 1);
    const int q = (lane & 1) ^ ((r >> 3) & 1);
    const long long row = a ? (long long)(m0 + r) : (long long)(n0 + r);
    const bool in = a ? (m0 + r < p.M) : (n0 + r < p.N);
    const long long e = plane * (a ? p.sa : p.sb) + row * (a ? p.lda : p.ldb) + 8 * q;
    voff[i] = in ? (uint32_t)(e * 2) : 0x7FFFFFF0u;
  }
  auto issue = [&](int stage, int kt) __attribute__((always_inline)) {
    const int soff = kt * B2K * 2;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int j = wave + 4 * i;
      auto* dst = (__attribute__((address_space(3))) void*)(lds + stage * STAGE3 * 2 + j * 1024);
      if (j < 12) __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, dst, 16, voff[i], soff, 0, 0);
      else __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, dst, 16, voff[i], soff, 0, 0);
    }
  };
  const int wm = wave >> 1, wn = wave & 1;
  const int r32 = lane & 31, h = lane >> 5;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = (p.K + B2K - 1) / B2K;
  issue(0, 0);
  if (nk > 1) issue(1, 1);
  if (nk > 1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  int st = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 2 < nk) issue(st == 0 ? 2 : st - 1, kt + 2);
    const __bf16* Ap = reinterpret_cast<const __bf16*>(lds) + st * STAGE3;
    const __bf16* Bp = Ap + 3 * P3;
    const Split3 b0 = ld3(Bp, wn * 64 + r32, h), b1 = ld3(Bp, wn * 64 + 32 + r32, h);
    const Split3 a0 = ld3(Ap, wm * 64 + r32, h);
    acc[0][0] = mfma_x6(a0, b0, acc[0][0]);
    acc[0][1] = mfma_x6(a0, b1, acc[0][1]);
    const Split3 a1 = ld3(Ap, wm * 64 + 32 + r32, h);
    acc[1][0] = mfma_x6(a1, b0, acc[1][0]);
    acc[1][1] = mfma_x6(a1, b1, acc[1][1]);
    if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    st = st == 2 ? 0 : st + 1;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + 32 * j + r32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < p.M && n < p.N) p.C[(long long)m * p.ldc + n] = acc[i][j][r];
      }
    }
}

// ---- variant 4: v1's 128 x 256 tile and wave layout, BK = 16, FOUR 36 KB stages with two stages
// of buffer_load ... lds in flight across each barrier (counted vmcnt: 36 pieces per stage, 5 for
// waves 0-3 and 4 for waves 4-7). Question: is v1 bound by the DMA latency its two stages expose?
constexpr int P4A = 128 * B2K, P4B = 256 * B2K;  // bf16 elements per A / B plane tile
constexpr int STAGE4 = 3 * P4A + 3 * P4B;        // 36 KB
constexpr int NST4 = 4;

template <int ASM>  // 0: builtin DMA (v4); 1: asm DMA (v7)
__global__ __launch_bounds__(NT, 1) void gemm_planes4_kernel(const PP p) {
  __shared__ __attribute__((aligned(16))) char lds[NST4 * STAGE4 * 2];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nx = (p.N + BN - 1) / BN, ny = (p.M + BM - 1) / BM;
  const int t = xcd_order(blockIdx.x + nx * blockIdx.y, nx * ny);
  const int GM = ny < 8 ? ny : 8, grp = t / (GM * nx), fm = grp * GM;
  const int gm = ny - fm < GM ? ny - fm : GM, tg = t - grp * GM * nx;
  const int m0 = (fm + tg % gm) * BM, n0 = (tg / gm) * BN;
  const rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0,
                                                      (int)((2 * p.sa + (long long)p.M * p.lda) * 2), 0x00020000);
  const rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0,
                                                      (int)((2 * p.sb + (long long)p.N * p.ldb) * 2), 0x00020000);
  // pieces j = wave + 8 i < 36: j < 12 A (plane j / 4, rows 32 (j % 4) ..), else B (plane
  // (j - 12) / 8, rows 32 ((j - 12) % 8) ..); lane l: row r0 + l / 2, slot l % 2 = quad ^ swz
  uint32_t voff[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int j = wave + 8 * i;
    const bool a = j < 12;
    const int jj = a ? j : j - 12;
    const int plane = a ? jj >> 2 : jj >> 3;
    const int r = (a ? jj & 3 : jj & 7) * 32 + (lane >> 1);
    const int q = (lane & 1) ^ ((r >> 3) & 1);
    const long long row = a ? (long long)(m0 + r) : (long long)(n0 + r);
    const bool in = j < 36 && (a ? (m0 + r < p.M) : (n0 + r < p.N));
    const long long e = plane * (a ? p.sa : p.sb) + row * (a ? p.lda : p.ldb) + 8 * q;
    voff[i] = in ? (uint32_t)(e * 2) : 0x7FFFFFF0u;
  }
  const bool five = wave < 4;  // wave-uniform: this wave moves 5 pieces per stage, else 4
  auto issue = [&](int stage, int kt) __attribute__((always_inline)) {
    const int soff = kt * B2K * 2;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int j = wave + 8 * i;
      if (j >= 36) break;
      if (j < 12) dma16<ASM>(rA, lds, stage * STAGE4 * 2 + j * 1024, voff[i], soff);
      else dma16<ASM>(rB, lds, stage * STAGE4 * 2 + j * 1024, voff[i], soff);
    }
  };
  // wait until at most `ahead` later stages of this wave's pieces are in flight
  auto wait_ahead = [&](int ahead) __attribute__((always_inline)) {
    if (five) {
      if (ahead >= 2) asm volatile("s_waitcnt vmcnt(10) lgkmcnt(0)" ::: "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(5) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    } else {
      if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
  };
  const int g = __builtin_amdgcn_readfirstlane(tid >> 8);
  const int wm = (wave >> 1) & 1, wn = wave & 1;
  const int r32 = lane & 31, h = lane >> 5;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = (p.K + B2K - 1) / B2K;
  for (int k = 0; k < 3 && k < nk; ++k) issue(k, k);
  wait_ahead(nk - 1 < 2 ? nk - 1 : 2);
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 3;
    if (kt + 3 < nk) issue((kt + 3) & 3, kt + 3);  // the buffer read one iteration ago
    const __bf16* Ap = reinterpret_cast<const __bf16*>(lds) + st * STAGE4;
    const __bf16* Bp = Ap + 3 * P4A;
    const int ra0 = wm * 64 + r32, rb0 = 128 * g + wn * 64 + r32;
    Split3 b0, b1, a0, a1;
    {
      const __bf16* q0 = Bp + off2(rb0, h);
      b0.h = *reinterpret_cast<const bf16x8*>(q0);
      b0.m = *reinterpret_cast<const bf16x8*>(q0 + P4B);
      b0.l = *reinterpret_cast<const bf16x8*>(q0 + 2 * P4B);
      const __bf16* q1 = Bp + off2(rb0 + 32, h);
      b1.h = *reinterpret_cast<const bf16x8*>(q1);
      b1.m = *reinterpret_cast<const bf16x8*>(q1 + P4B);
      b1.l = *reinterpret_cast<const bf16x8*>(q1 + 2 * P4B);
      const __bf16* q2 = Ap + off2(ra0, h);
      a0.h = *reinterpret_cast<const bf16x8*>(q2);
      a0.m = *reinterpret_cast<const bf16x8*>(q2 + P4A);
      a0.l = *reinterpret_cast<const bf16x8*>(q2 + 2 * P4A);
    }
    acc[0][0] = mfma_x6(a0, b0, acc[0][0]);
    acc[0][1] = mfma_x6(a0, b1, acc[0][1]);
    {
      const __bf16* q3 = Ap + off2(ra0 + 32, h);
      a1.h = *reinterpret_cast<const bf16x8*>(q3);
      a1.m = *reinterpret_cast<const bf16x8*>(q3 + P4A);
      a1.l = *reinterpret_cast<const bf16x8*>(q3 + 2 * P4A);
    }
    acc[1][0] = mfma_x6(a1, b0, acc[1][0]);
    acc[1][1] = mfma_x6(a1, b1, acc[1][1]);
    // stage kt + 1 must have landed; stages kt + 2, kt + 3 (if issued) stay in flight
    const int issued_ahead = (nk - 1 - kt) < 3 ? (nk - 1 - kt) : 3;  // stages after kt issued
    wait_ahead(issued_ahead - 1);
    __builtin_amdgcn_s_barrier();
  }
  float* Cs = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ml = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int nl = 128 * g + wn * 64 + j * 32 + r32;
        Cs[ml * BN + nl] = acc[i][j][r];
      }
  __syncthreads();
  const int nl = tid & (BN - 1);
  if (n0 + nl < p.N)
    for (int ml = tid >> 8; ml < BM && m0 + ml < p.M; ml += 2) p.C[(long long)(m0 + ml) * p.ldc + n0 + nl] = Cs[ml * BN + nl];
}

// reference: C = sum_k (A0+A1+A2)(B0+B1+B2) in double (naive)
__global__ void ref_kernel(const PP p, double* Cr) {
  const int m = blockIdx.y, n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= p.N) return;
  double s = 0;
  for (int k = 0; k < p.K; ++k) {
    double a = 0, b = 0;
    for (int pl = 0; pl < 3; ++pl) {
      a += (double)(float)p.A[pl * p.sa + (long long)m * p.lda + k];
      b += (double)(float)p.B[pl * p.sb + (long long)n * p.ldb + k];
    }
    s += a * b;
  }
  Cr[(long long)m * p.N + n] = s;
}

static unsigned short f2bf(float x) {  // round to nearest even
  unsigned u;
  std::memcpy(&u, &x, 4);
  u += 0x7FFF + ((u >> 16) & 1);
  return (unsigned short)(u >> 16);
}
static float bf2f(unsigned short b) {
  unsigned u = (unsigned)b << 16;
  float x;
  std::memcpy(&x, &u, 4);
  return x;
}
static void split3(float x, unsigned short* o) {
  o[0] = f2bf(x);
  const float r1 = x - bf2f(o[0]);
  o[1] = f2bf(r1);
  o[2] = f2bf(r1 - bf2f(o[1]));
}

int main(int argc, char** argv) {
  struct Shape {
    int M, N, K;
    const char* what;
  } shapes[] = {
      {2048, 2048, 2048, "square 2048"},
      {4096, 4096, 4096, "square 4096"},
      {1536, 13824, 8064, "wgrad audio L0 conv2 (M=Cout, N=3Cin, K=B T)"},
      {2048, 9216, 4032, "wgrad audio L1"},
      {3072, 18432, 2016, "wgrad audio L2"},
      {1024, 6144, 8064, "wgrad up3 conv1"},
      {2048, 8064, 4608, "conv fwd L1 audio (M=Cout, N=B T, K=3 Cin)"},
      {1536, 8064, 4608, "conv fwd L0 audio"},
  };
  const bool check = argc > 1 && atoi(argv[1]) != 0;
  const int only = argc > 2 ? atoi(argv[2]) : 0;  // one variant
  for (const Shape& s : shapes) {
    const int Kp = (s.K + 31) / 32 * 32;
    PP p{};
    p.M = s.M, p.N = s.N, p.K = Kp, p.lda = Kp, p.ldb = Kp, p.ldc = s.N;
    p.sa = (long long)s.M * Kp, p.sb = (long long)s.N * Kp;
    std::vector<unsigned short> ha(3 * p.sa), hb(3 * p.sb);
    srand(1);
    for (long long i = 0; i < (long long)s.M * Kp; ++i) {
      unsigned short o[3];
      split3((float)((double)rand() / RAND_MAX * 2.0 - 1.0), o);
      for (int pl = 0; pl < 3; ++pl) ha[pl * p.sa + i] = o[pl];
    }
    for (long long i = 0; i < (long long)s.N * Kp; ++i) {
      unsigned short o[3];
      split3((float)((double)rand() / RAND_MAX * 2.0 - 1.0), o);
      for (int pl = 0; pl < 3; ++pl) hb[pl * p.sb + i] = o[pl];
    }
    __bf16 *da, *db;
    float* dc;
    CK(hipMalloc(&da, ha.size() * 2));
    CK(hipMalloc(&db, hb.size() * 2));
    CK(hipMalloc(&dc, (size_t)s.M * s.N * 4));
    CK(hipMemcpy(da, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
    p.A = da, p.B = db, p.C = dc;
   for (int var = 1; var <= 12; ++var) {
    if (var == 2 || var == 3 || var == 4 || var == 6 || var == 7) continue;  // measured: profiles/r05/gemm_planes_micro*.txt, profiles/r06/
    if (only && var != only) continue;
    dim3 grid = dim3((s.N + BN - 1) / BN, (s.M + BM - 1) / BM);
    auto launch = [&]() {
      if (var == 1) hipLaunchKernelGGL(gemm_planes_kernel<0>, grid, dim3(NT), 0, 0, p);
      else if (var == 5) hipLaunchKernelGGL(gemm_planes_kernel<1>, grid, dim3(NT), 0, 0, p);
      else if (var == 6) hipLaunchKernelGGL(gemm_planes_kernel<2>, grid, dim3(NT), 0, 0, p);
      else if (var == 4) hipLaunchKernelGGL(gemm_planes4_kernel<0>, grid, dim3(NT), 0, 0, p);
      else if (var == 7) hipLaunchKernelGGL(gemm_planes4_kernel<1>, grid, dim3(NT), 0, 0, p);
      else if (var == 8) hipLaunchKernelGGL((gemm_planes_x_kernel<true, false, false>), grid, dim3(NT), 0, 0, p);
      else if (var == 9) hipLaunchKernelGGL((gemm_planes_x_kernel<false, true, false>), grid, dim3(NT), 0, 0, p);
      else if (var == 10) hipLaunchKernelGGL((gemm_planes_x_kernel<true, true, false>), grid, dim3(NT), 0, 0, p);
      else if (var == 11) hipLaunchKernelGGL((gemm_planes_x_kernel<false, false, true>), grid, dim3(NT), 0, 0, p);
      else if (var == 12) hipLaunchKernelGGL((gemm_planes_x_kernel<false, true, true>), grid, dim3(NT), 0, 0, p);
    };
    CK(hipMemset(dc, 0, (size_t)s.M * s.N * 4));
    launch();
    CK(hipDeviceSynchronize());
    if (check) {
      double* dr;
      CK(hipMalloc(&dr, (size_t)s.M * s.N * 8));
      hipLaunchKernelGGL(ref_kernel, dim3((s.N + 255) / 256, s.M), dim3(256), 0, 0, p, dr);
      CK(hipDeviceSynchronize());
      std::vector<double> r((size_t)s.M * s.N);
      std::vector<float> c((size_t)s.M * s.N);
      CK(hipMemcpy(r.data(), dr, r.size() * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(c.data(), dc, c.size() * 4, hipMemcpyDeviceToHost));
      double worst = 0, scale = 0;
      for (size_t i = 0; i < r.size(); ++i) {
        worst = fmax(worst, fabs(c[i] - r[i]));
        scale = fmax(scale, fabs(r[i]));
      }
      printf("check v%d %-45s max|err| %.3e of max|C| %.3e (%.2e)\n", var, s.what, worst, scale, worst / scale);
      CK(hipFree(dr));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 50;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    const double tf = 2.0 * s.M * s.N * s.K / (ms * 1e-3) / 1e12;
    printf("v%d %-50s M %5d N %5d K %5d tiles %4d  %.3f ms  %.1f TF/s fp32-equiv (%.3f of 416.7)\n", var,
           s.what, s.M, s.N, s.K, grid.x * grid.y, ms, tf, tf / 416.7);
    if (var == 8 || var == 10) {  // in-kernel clock of the last launch: median over workgroups of dmemtime/drealtime
      const int nwg = (int)(grid.x * grid.y) < 65536 ? (int)(grid.x * grid.y) : 65536;
      std::vector<unsigned long long> h(4 * nwg);
      CK(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_clk), h.size() * 8));
      std::vector<double> f;
      for (int w = 0; w < nwg; ++w) {
        const double dt = (double)(h[4 * w + 3] - h[4 * w + 1]);
        if (dt > 0) f.push_back((double)(h[4 * w + 2] - h[4 * w]) / dt * 0.1);  // GHz (realtime 100 MHz)
      }
      std::sort(f.begin(), f.end());
      const double ghz = f.empty() ? 0 : f[f.size() / 2];
      printf("   clock %.3f GHz (median of %zu workgroups): ceiling at that clock %.1f TF/s, this kernel %.3f of it\n",
             ghz, f.size(), 416.7 * ghz / 2.4, tf / (416.7 * ghz / 2.4));
    }
   }
    CK(hipFree(da));
    CK(hipFree(db));
    CK(hipFree(dc));
  }
  return 0;
}
