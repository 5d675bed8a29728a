// Implicit-GEMM conv/linear kernels on gfx950: fp32 products on the bf16 matrix cores
// (v_mfma_f32_32x32x16_bf16, operands split exactly into three bf16 planes, see below).
//
// One kernel body serves every dense contraction of PerformanceNet (model/model.py):
//   forward  Conv1d k3 p1 (model.py:14-22), Linear (model.py:98-99, NCL = 1-tap conv),
//            ConvTranspose1d s2 p1 (model.py:24-31) as two sub-pixel phases,
//            ConvTranspose1d k3 s1 p1 (lastconv, model.py:242)
//   dgrad    the same layers' input gradients (stride-1 or stride-2 gathers over dY)
//   wgrad    weight gradients: sum over (batch, time) of dY x input
// Inputs are read through "virtual concat" descriptors (two channel slabs with time
// offsets), which is how torch.cat + crop_and_concat (model.py:71-78, 103) are fused
// away, and the epilogue applies alpha/bias/activation/dropout and routes rows to two
// destinations (the concat split of an input gradient) with an optional ReLU/dropout
// gate (DenseConcat backward).
//
// Tile: 128x128 block, BK=32, 256 threads = 4 waves in 2x2, each wave 64x64 = 2x2
// MFMA 32x32 tiles. Global loads are register-staged two tiles ahead; each loaded element is
// split once into three bf16 planes when it is stored to LDS (see pl_off).
//
// Operands are fetched with raw buffer loads (32-bit byte offsets into a descriptor per
// tensor): an element outside the tensor's valid ranges gets an out-of-range offset and the
// hardware returns 0, so the loaders have no branches and no post-load selects. fp32 MFMA
// shares the SIMD's f32 datapath with VALU (rocprofv3: SQ_VALU_MFMA_COEXEC_CYCLES = 0), so
// every loader VALU instruction costs MFMA issue time: the per-element index work is kept
// wave-uniform (scalar) wherever the mapping allows it.
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 32, NTHR = 256;

constexpr uint32_t OOB = 0x7FFFFFF0u;  // byte offset past every descriptor's num_records
constexpr int MAXCLS = 8;              // wgrad K classes

typedef __amdgpu_buffer_rsrc_t rsrc_t;

// fp32 products on the bf16 matrix cores ("bf16x6"): every fp32 operand is split exactly into
// three bf16 pieces x = x0 + x1 + x2 (round-to-nearest at each step: the residual x - x0 has at
// most 16 significant bits and x1 - r1 at most 8, so the split loses nothing for normal
// values), and a . b = sum of the six products xi yj with i + j <= 2: the three dropped terms
// are below 2^-24 relative, the size of the fp32 path's own rounding. Each bf16 x bf16
// product is exact and v_mfma_f32_32x32x16_bf16 accumulates in fp32, so the result carries
// fp32-level error (tests/test_gpu_kernels.py bounds it with the fp32 tolerances) at 6 MFMAs
// of 32 cycles per 16-deep k step instead of 8 fp32 MFMAs of 64 cycles: 2.7x less matrix-
// core time. (Rounds 1-2 ran v_mfma_f32_32x32x2_f32 on fp32 tiles and then split after every
// LDS read; both were measured slower and removed: DESIGN.md, GEMM design.)
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
struct Split3 {
  bf16x8 h, m, l;
};

// The split happens once per element, when a loaded tile is stored: A and B sit in LDS as
// three bf16 planes (hi, mid, lo) of [row][k]. The 6 planes (48 KB) take ONE buffer (the 64 KB
// epilogue tile aliases it), so two workgroups fit per CU: the tile loop stores, syncs, runs the
// MFMAs, syncs, and the other workgroup on the CU fills the store phase.
// Plane rows are 64 B (32 bf16, no padding) with the four 16-byte quads of row r XOR-swizzled by
// swz(r) = r2 | (r1 ^ r3) << 1 (r_i: bit i of r). The banking rules (MI355X_MICROARCH.md, LDS
// table) it satisfies: a ds_read_b128 fragment read (16-row lane groups {0-3, 12-15, 20-27} and
// {4-11, 16-19, 28-31}, 64 banks) and a k-major ds_write_b64 (16 contiguous lanes = 2 rows, 32
// banks) each touch every bank once, and so does a row-major ds_write_b128 (8 contiguous lanes =
// 8 rows, 32 banks: rows of one parity need distinct swizzles). The round-3 swizzle (r >> 2) & 3
// made that last one 2-way (PMC: 20 % of conv and 33 % of dgrad LDS cycles were conflicts,
// profiles/r04/pmc_gemm_m4_summary.txt). The row-major writes pair two k quads into one 16-byte
// store per plane (their unit order, rm_quad, makes a thread's quads adjacent).
constexpr int LDKB = BK;
constexpr int PLANE = BM * LDKB;  // bf16 elements per plane (BM == BN)
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int pl_swz(int row) {
  return ((row >> 2) & 1) | (((row >> 1) ^ (row >> 3)) & 1) << 1;
}
__device__ __forceinline__ int pl_off(int row, int q) {  // element offset of (row, 16-B quad q)
  return row * LDKB + 8 * (q ^ pl_swz(row));
}

struct Bf3 {
  __bf16 h, m, l;
};
__device__ __forceinline__ Bf3 split1(float x) {
  const __bf16 b0 = (__bf16)x;
  const float r1 = x - (float)b0;
  const __bf16 b1 = (__bf16)r1;
  return Bf3{b0, b1, (__bf16)(r1 - (float)b1)};
}

// 4 consecutive k (k0 = 4 c8) of one row: three 8-byte stores (PS: elements per plane)
template <int PS = PLANE>
__device__ __forceinline__ void split_store4(__bf16* plane0, int row, int c8, const f32x4 v) {
  bf16x4 hi, mid, lo;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const Bf3 t = split1(v[i]);
    hi[i] = t.h;
    mid[i] = t.m;
    lo[i] = t.l;
  }
  const int off = pl_off(row, c8 >> 1) + 4 * (c8 & 1);
  *reinterpret_cast<bf16x4*>(plane0 + off) = hi;
  *reinterpret_cast<bf16x4*>(plane0 + PS + off) = mid;
  *reinterpret_cast<bf16x4*>(plane0 + 2 * PS + off) = lo;
}

// 8 consecutive k (quad q) of one row from two units: three 16-byte stores
template <int PS = PLANE>
__device__ __forceinline__ void split_store8(__bf16* plane0, int row, int q, const f32x4 v0,
                                             const f32x4 v1) {
  bf16x8 hi, mid, lo;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const Bf3 t = split1(i < 4 ? v0[i] : v1[i - 4]);
    hi[i] = t.h;
    mid[i] = t.m;
    lo[i] = t.l;
  }
  const int off = pl_off(row, q);
  *reinterpret_cast<bf16x8*>(plane0 + off) = hi;
  *reinterpret_cast<bf16x8*>(plane0 + PS + off) = mid;
  *reinterpret_cast<bf16x8*>(plane0 + 2 * PS + off) = lo;
}

template <int PS = PLANE>
__device__ __forceinline__ Split3 ld_planes(const __bf16* base, int row, int q) {
  const __bf16* p = base + pl_off(row, q);
  Split3 s;
  s.h = *reinterpret_cast<const bf16x8*>(p);
  s.m = *reinterpret_cast<const bf16x8*>(p + PS);
  s.l = *reinterpret_cast<const bf16x8*>(p + 2 * PS);
  return s;
}

// Row-major tile units: thread (row, kw) holds 4-float k units rm_quad(kw, u) = 4 kw + u,
// u = 0..3 (a thread's units adjacent, stored to the planes in pairs).
__device__ __forceinline__ constexpr int rm_quad(int kw, int u) { return 4 * kw + u; }

constexpr int LDS_FLOATS = BM * BN;  // the 64 KB epilogue tile; the 48 KB of planes alias it

// acc += a . b over one 16-deep k step, smallest products first
__device__ __forceinline__ f32x16 mfma_x6(const Split3& a, const Split3& b, f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.l, b.h, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.l, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.m, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.h, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.m, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.h, acc, 0, 0, 0);
  return acc;
}

struct GP {
  int M, N, K, nk, splitk;
  long long nA, nP, nx0, nx1;  // elements addressable through each operand descriptor
  int dual;                    // second input source present
  int nbT, nb0;                // conv: 32-deep K tiles per tap / of source 0 within a tap
  // conv A operand
  const float* A;
  long long sAm, sAc, sAt;
  int a_mode;  // 0: k-scalar, 1: k-vector (float4), 2: m-major
  // wgrad A operand (P = dY or X, time contiguous)
  const float* P;
  long long sPb;
  int sPc, Tk;
  int Tp, lo, span;  // padded time axis; valid input times [lo, lo + span) of the single source
  int ncls;          // K classes of the wgrad tile order (see the main loop)
  int cstart[MAXCLS + 1], ct0[MAXCLS], ccnt[MAXCLS], cmask[MAXCLS];
  // virtual input (B operand source)
  const float* x0;
  long long sb0;
  int sc0, C0, T0, off0;
  const float* x1;
  long long sb1;
  int sc1, T1, off1, C1;
  int Tv, ta, tb, tg;
  int Tn;
  // conv epilogue
  int ostride, ophase;
  float* y0;
  long long yb0;
  int yc0, M0, yT0, yoff0;
  const float* gt0;
  float gs0;
  float* y1;
  long long yb1;
  int yc1, yT1, yoff1;
  const float* gt1;
  float gs1;
  float alpha;
  const float* bias;
  int act;
  float drop_p;
  unsigned long long seed;
  const unsigned long long* seed_dev;  // nullable: key seed = seed + *seed_dev
  // wgrad epilogue
  float* out;
  long long ldo, ldc, ldt;  // column of (c, tap) = c * ldc + tap * ldt
  int taps, ocustom;
  float inv_taps;
  float scale;
  int accumulate;
  // split-K slab
  float* ws;
  int wide;  // conv / dgrad on the 128 x 256 kernel (gemm_w_kernel)
  int wvec;  // wgrad: dwordx4 loads in unmasked unit-stride K classes (MST_WG_VEC=0: dword)
  // stream-K (sk_L > 0): the grid's G workgroups each run sk_L consecutive iterations of the
  // flattened (tile, 32-deep K tile) space of sk_I = tiles * nk iterations
  long long sk_L, sk_I;
  // pre-split operand planes (gemm_p_kernel): 3 bf16 planes each, [rows][pld] (k contiguous)
  const __bf16* pA;
  const __bf16* pB;
  long long psa, psb;  // plane strides (elements)
  int pld;             // row stride = padded K (a multiple of BK)
  int slab4;  // split-K slabs stored as dwordx4 rows (N % 4 == 0, M N < 2^29; store_slab4)
  int b2;     // weight-gradient B planes in two copies (build_wgrad_planes); bC: channels
  int bC;
};

// Tile-order index -> (M tile, N tile): runs of GM M-tiles x all N-tiles, M fastest within a
// run, so a contiguous range of indices is a near-square block of tiles (8 x 8 when it holds
// 64) whose A and B panels are re-read from one L2.
__device__ __forceinline__ void tile_of(int t2, int nx, int ny, int& m_t, int& n_t) {
  const int GM = ny < 8 ? ny : 8;
  const int grp = t2 / (GM * nx);
  const int fm = grp * GM;
  const int gm = ny - fm < GM ? ny - fm : GM;
  const int tg = t2 - grp * GM * nx;
  m_t = fm + tg % gm;
  n_t = tg / gm;
}

// XCD-aware workgroup numbering. Workgroups are dealt round-robin over the 8 XCDs (linear id
// % 8), each with its own L2: renumber so every XCD runs one contiguous range of indices.
__device__ __forceinline__ int xcd_order(int w, int W) {
  const int q = W >> 3, r = W & 7, xcd = w & 7;
  return xcd * q + min(xcd, r) + (w >> 3);
}

// bias value bm = p.bias[m] passed in (loaded ahead by the caller: a load inside this per-element
// path, behind its branches, makes the compiler wait for it element by element)
// element (m, n = b Tn + t) with (b, t) known
__device__ __forceinline__ void conv_store_bt(const GP& p, int m, int b, int t, float v, float bm) {
  v *= p.alpha;
  if (p.bias) v += bm;
  if (p.act == MST_ACT_RELU) v = fmaxf(v, 0.f);
  else if (p.act == MST_ACT_LRELU) v = v > 0.f ? v : 0.01f * v;
  int to = t * p.ostride + p.ophase;
  if (m < p.M0) {
    int ts = to + p.yoff0;
    if ((unsigned)ts >= (unsigned)p.yT0) return;
    long long idx = (long long)b * p.yb0 + (long long)m * p.yc0 + ts;
    if (p.drop_p > 0.f) {
      const unsigned long long sd = p.seed + (p.seed_dev ? *p.seed_dev : 0ull);
      uint32_t h = mst_hash32(sd, (unsigned long long)idx);
      v = (h >= (uint32_t)(p.drop_p * 4294967296.0f)) ? v * (1.f / (1.f - p.drop_p)) : 0.f;
    }
    if (p.gt0) v = p.gt0[idx] > 0.f ? v * p.gs0 : 0.f;
    p.y0[idx] = v;
  } else {
    int mm = m - p.M0;
    int ts = to + p.yoff1;
    if ((unsigned)ts >= (unsigned)p.yT1) return;
    long long idx = (long long)b * p.yb1 + (long long)mm * p.yc1 + ts;
    if (p.gt1) v = p.gt1[idx] > 0.f ? v * p.gs1 : 0.f;
    p.y1[idx] = v;
  }
}

__device__ __forceinline__ void conv_store_b(const GP& p, int m, int n, float v, float bm) {
  if (m >= p.M || n >= p.N) return;
  const int b = n / p.Tn;
  conv_store_bt(p, m, b, n - b * p.Tn, v, bm);
}

__device__ __forceinline__ void conv_store(const GP& p, int m, int n, float v) {
  conv_store_b(p, m, n, v, (p.bias && m < p.M) ? p.bias[m] : 0.f);
}

__device__ __forceinline__ void wgrad_store(const GP& p, int m, int n, float v) {
  if (m >= p.M || n >= p.N) return;
  long long col = n;  // n = c * taps + tap: the column in the torch layout
  if (p.ocustom) {    // e.g. tap-major weights: column = c * ldc + tap * ldt
    const int c = (int)(((float)n + 0.5f) * p.inv_taps);  // exact for n < 2^22
    col = (long long)c * p.ldc + (long long)(n - c * p.taps) * p.ldt;
  }
  float* o = p.out + (long long)m * p.ldo + col;
  v *= p.scale;
  if (p.accumulate) v += *o;
  *o = v;
}

// Value select: `c ? x : y` on two lvalues (lambda captures, kernarg fields) is an lvalue, and
// the compiler implements it by taking both addresses, which moves the operands to scratch.
template <class T>
__device__ __forceinline__ T sel(bool c, T x, T y) {
  return c ? x : y;
}

__device__ __forceinline__ rsrc_t mk_rsrc(const float* ptr, long long n) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)ptr, (short)0, (int)(n * 4), 0x00020000);
}

__device__ __forceinline__ float ldb(rsrc_t r, uint32_t voff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, 0, 0));
}

__device__ __forceinline__ f32x4 ldb4(rsrc_t r, uint32_t voff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, 0, 0));
}

// voffset (per lane, VGPR) + soffset (wave-uniform, SGPR): the per-element part of a conv
// operand address is scalar, so these loads cost no VALU.
__device__ __forceinline__ float ldbs(rsrc_t r, uint32_t voff, int soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, soff, 0));
}

__device__ __forceinline__ f32x4 ldbs4(rsrc_t r, uint32_t voff, int soff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, soff, 0));
}

// One pass over K tiles [kt0, kt1) of output tile (m_t, n_t), then the epilogue: the final
// values (direct), split-K slab `split`, or (slab != nullptr) a stream-K partial tile.
template <int TAPS, bool WG, int AMODE, bool DUAL>
__device__ __forceinline__ void tile_pass(const GP& p, float* lds, int m_t,
                                          int n_t, int kt0, int kt1, int split, float* slab,
                                          int tid) {
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int n0 = n_t * BN;
  const int m0 = m_t * BM;

  // Two unit mappings of a 128-row x 32-k tile onto 256 threads, 4 units of 4 consecutive k:
  //   KM ("k-major"): row = (tid>>3) + 32u, k quad = tid&7 -> 8 lanes run along k
  //   RM ("row-major"): row = tid&127, k quads rm_quad(kw, u) -> lanes run along rows; k is
  //                     wave-uniform (kw = tid>>7 via readfirstlane), so its decode is scalar
  // both are split into the bf16 planes at the LDS store (pl_off).
  // A: AMODE 1 (k-contiguous, float4) and 0 (k-scalar) use KM; AMODE 2 (m-contiguous) RM.
  // B: conv/dgrad (n = time, contiguous) RM; wgrad (k = time) KM.
  // k-major unit u of this thread: row km_r(u), 4-float k unit km_q(u) (8 lanes along k per row)
  auto km_r = [&](int u) __attribute__((always_inline)) { return (tid >> 3) + 32 * u; };
  auto km_q = [&](int u) __attribute__((always_inline)) { return tid & 7; };
  const int rm_row = tid & 127;
  const int kw = __builtin_amdgcn_readfirstlane(tid >> 7);

  f32x4 ra[2][4], rb[2][4];  // two register stages: tile k+2 loads while k+1 waits

  // ------------------------------------------------------------ loaders
  const rsrc_t rX0 = mk_rsrc(p.x0, p.nx0);
  const rsrc_t rA = mk_rsrc(WG ? p.P : p.A, WG ? p.nP : p.nA);

  // per-lane constants
  uint32_t rowA[4];
  int tinb = 0;
  uint32_t colb0 = 0, colb1 = 0;
  // wgrad: per-element offsets of the current K class (set per class, see the main loop)
  uint32_t vA[4], vB[4][4];
  if constexpr (!WG) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int m = m0 + (AMODE == 2 ? rm_row : km_r(u));
      // KM: the lane's k unit is a fixed channel offset within every tile
      rowA[u] = m < p.M ? (uint32_t)(m * p.sAm + (AMODE == 2 ? 0 : 4 * km_q(u) * p.sAc)) * 4u : OOB;
    }
    const int n = n0 + rm_row;
    const int bb = n / p.Tn;
    const int tt = n - bb * p.Tn;
    tinb = n < p.N ? p.ta * tt + p.tb : -(1 << 29);  // invalid column: every tap out of range
    colb0 = (uint32_t)(bb * p.sb0) * 4u;
    colb1 = DUAL ? (uint32_t)(bb * p.sb1) * 4u : 0u;
  }
  // wgrad K order: k = (b, t) with the time axis padded to Tp (16, or a multiple of 32), so
  // a 32-deep tile is one batch row (or two 16-halves when Tp = 16). Unit u's k quad (4
  // consecutive t) sits at time tl(u) of batch b + bd(u).
  auto tl = [&](int u) __attribute__((always_inline)) {
    const int q = km_q(u);
    return p.Tp == 16 && q >= 4 ? 4 * q - 16 : 4 * q;
  };
  auto bd = [&](int u) __attribute__((always_inline)) { return p.Tp == 16 && km_q(u) >= 4 ? 1 : 0; };
  // Per-element offsets of one wgrad K class: every tile of the class shares the time offset
  // t0 - t0ref (a scalar soffset), so range checks against the input and the padding are
  // evaluated once per class here and the tile loop has no per-element work. Invalid elements
  // get the OOB offset (hardware zero).
  auto wg_class_setup = [&](int t0ref, bool masked) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int m = m0 + km_r(u);
      const int n = n0 + km_r(u);
      const int c = n / TAPS;  // N order n = c * taps + tap for every output layout
      const int tap = n - c * TAPS;
      const int tlb = tl(u), bdl = bd(u);
      const int abase = m * p.sPc + bdl * (int)p.sPb + t0ref + tlb;
      const int tin0 = p.ta * (t0ref + tlb) + p.tb + p.tg * tap;  // input time at i = 0
      const int bbase = c * p.sc0 + bdl * (int)p.sb0 + tin0 + p.off0;
      // A (P) is read unmasked: padded times read finite neighbours (or OOB zeros) and are
      // multiplied by B elements masked to zero there.
      vA[u] = m < p.M ? (uint32_t)abase * 4u : OOB;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int tin = tin0 + p.ta * i;
        const bool bok = n < p.N && (!masked || ((unsigned)(tin - p.lo) < (unsigned)p.span &&
                                                 t0ref + tlb + i < p.Tk));
        vB[u][i] = bok ? (uint32_t)(bbase + p.ta * i) * 4u : OOB;
      }
    }
  };

  // Conv K order is tap-major, k = tap * Cp + (source block, channel), each source's channels
  // padded to a multiple of BK: a 32-deep tile has ONE tap and ONE source, so the tile decode
  // is scalar, the lane's time index is one VGPR per tile, and every element offset is a
  // wave-uniform soffset. Padded channels read through a zero-length descriptor (B = 0).
  auto load_tile = [&](auto S, int kt, int tap, int blk, auto V) __attribute__((always_inline)) {
    constexpr int st_ = decltype(S)::value;
    constexpr bool vec = decltype(V)::value;
    (void)kt;
    if constexpr (!WG) {
      const bool s1 = DUAL && blk >= p.nb0;
      const int cb = (s1 ? blk - p.nb0 : blk) * BK;  // first channel of the tile in its source
      const int ci = cb + sel(s1, p.C0, 0);           // ... in the concatenated input
      const int Cs = sel(s1, p.C1, p.C0);
      // ---------------- A ----------------
      const int sA = (ci * p.sAc + tap * p.sAt) * 4;
      if constexpr (AMODE == 1) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          ra[st_][u] = ldbs4(rA, rowA[u], sA);
        }
      } else if constexpr (AMODE == 0) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int i = 0; i < 4; ++i) ra[st_][u][i] = ldbs(rA, rowA[u], sA + i * p.sAc * 4);
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            ra[st_][u][i] = ldbs(rA, rowA[0], sA + (4 * rm_quad(kw, u) + i) * p.sAc * 4);
      }
      // ---------------- B: X(b, c, a*t + beta + g*tap), column per lane ----------------
      const int tin = tinb + p.tg * tap;
      const int ts = tin + sel(s1, p.off1, p.off0);
      const bool ok = ((unsigned)tin < (unsigned)p.Tv) & ((unsigned)ts < (unsigned)sel(s1, p.T1, p.T0));
      const uint32_t lo = ok ? sel(s1, colb1, colb0) + (uint32_t)ts * 4u : OOB;
      // source descriptor built from scalars (selecting between descriptors spills them)
      const float* xs = sel(DUAL && s1, p.x1, p.x0);
      const long long ns = sel(DUAL && s1, p.nx1, p.nx0);
      const int scb = sel(s1, p.sc1, p.sc0) * 4;
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = cb + 4 * rm_quad(kw, u) + i;  // wave-uniform
          rb[st_][u][i] = ldbs(mk_rsrc(xs, c < Cs ? ns : 0), lo, c * scb);
        }
    } else {
      // wgrad tile of batch row b = tap at time t0ref + 32 * blk: one scalar soffset per operand
      const int sA = (tap * (int)p.sPb + BK * blk) * 4;
      const int sB = (tap * (int)p.sb0 + p.ta * BK * blk) * 4;
      if constexpr (vec) {
        // unmasked class, unit stride: each unit's 4 k are 4 consecutive floats of one row, all
        // in range (an interior tile lies inside its row), so one dwordx4 per unit (dword-aligned;
        // a partially out-of-range x4 only occurs in prefetches past the class, never consumed)
#pragma unroll
        for (int u = 0; u < 4; ++u) ra[st_][u] = ldbs4(rA, vA[u], sA);
#pragma unroll
        for (int u = 0; u < 4; ++u) rb[st_][u] = ldbs4(rX0, vB[u][0], sB);
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int i = 0; i < 4; ++i) ra[st_][u][i] = ldbs(rA, vA[u], sA + 4 * i);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int i = 0; i < 4; ++i) rb[st_][u][i] = ldbs(rX0, vB[u][i], sB);
      }
    }
  };

  auto store_tile = [&](auto S) __attribute__((always_inline)) {
    constexpr int st = decltype(S)::value;
    __bf16* Ap = reinterpret_cast<__bf16*>(lds);
    __bf16* Bp = Ap + 3 * PLANE;
    if constexpr (AMODE == 2 && !WG) {  // quads 4 kw + u: pairs (0, 1), (2, 3) are adjacent
#pragma unroll
      for (int u = 0; u < 4; u += 2) split_store8(Ap, rm_row, 2 * kw + u / 2, ra[st][u], ra[st][u + 1]);
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) split_store4(Ap, km_r(u), km_q(u), ra[st][u]);
    }
    if constexpr (WG) {
#pragma unroll
      for (int u = 0; u < 4; ++u) split_store4(Bp, km_r(u), km_q(u), rb[st][u]);
    } else {
#pragma unroll
      for (int u = 0; u < 4; u += 2) split_store8(Bp, rm_row, 2 * kw + u / 2, rb[st][u], rb[st][u + 1]);
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int r32 = lane & 31;
  const int h = lane >> 5;

  // Branch-free main loop: the prefetch of tile k+1 is issued unconditionally (past the
  // end of K every element resolves to the zero block) so no control-flow join forces a
  // vmcnt(0) between the prefetch and this tile's MFMAs.
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  auto mfma_tile = [&]() __attribute__((always_inline)) {
    const __bf16* Ap = reinterpret_cast<const __bf16*>(lds);
    const __bf16* Bp = Ap + 3 * PLANE;
    // 32x32x16 bf16 operand layout: lane (r32, h) supplies row r32, k = 16 s + 8 h + [0, 8)
    const int ra0 = wm * 64 + r32, rb0 = wn * 64 + r32;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const Split3 b0 = ld_planes(Bp, rb0, 2 * s + h), b1 = ld_planes(Bp, rb0 + 32, 2 * s + h);
      {
        const Split3 a0 = ld_planes(Ap, ra0, 2 * s + h);
        acc[0][0] = mfma_x6(a0, b0, acc[0][0]);
        acc[0][1] = mfma_x6(a0, b1, acc[0][1]);
      }
      {
        const Split3 a1 = ld_planes(Ap, ra0 + 32, 2 * s + h);
        acc[1][0] = mfma_x6(a1, b0, acc[1][0]);
        acc[1][1] = mfma_x6(a1, b1, acc[1][1]);
      }
    }
  };

  // Pipeline: one LDS buffer of planes + two register stages. Iteration k issues the global
  // loads of tile k+2, runs tile k's MFMAs from LDS, syncs, then splits and stores tile k+1
  // (loaded one iteration earlier, so its latency is covered by a full tile of MFMAs); the other
  // workgroup on the CU runs its MFMAs while this one stores. Loads past the end are harmless
  // (bounded buffer loads) and never consumed.
  // run(): one pipelined pass over tiles [kb, ke) starting at scalar decode (tap, blk).
  //   conv : (tap, source block) of a tap-major K
  //   wgrad: (batch row b, tile index j within the class), `per` tiles per row
  auto run = [&](int kb, int ke, int tap, int blk, int per, auto V) __attribute__((always_inline)) {
    constexpr bool vec = decltype(V)::value;
    auto advance = [&]() __attribute__((always_inline)) {
      if (++blk == per) {
        blk = 0;
        tap += (WG && p.Tp == 16) ? 2 : 1;
      }
    };
    load_tile(I0{}, kb, tap, blk, V);
    advance();
    load_tile(I1{}, kb + 1, tap, blk, V);
    advance();
    store_tile(I0{});
    __syncthreads();
    auto step = [&](auto S, int kt) __attribute__((always_inline)) {
      constexpr int sb = decltype(S)::value;
      load_tile(S, kt + 2, tap, blk, V);
      advance();
      mfma_tile();
      // Interleave the next-tile global loads with this tile's MFMAs, spread evenly over the 48
      // MFMAs (sched_group_barrier). Issued as a block above the MFMAs they cost 15-25 % of the
      // GEMM (A/B: conv fwd +5-10 %, dgrad +9-13 %, wgrad +15-25 %); left to the scheduler
      // they sink next to their wait. Evenly spread instead of one per MFMA from the first
      // (round 4): wgrad +1.5-2.4 % (gemm_micro), the step +0.6 % (profiles/r04/
      // gemm_micro_m14_*); s_setprio 1 around the MFMAs lost 8 %.
      constexpr int NV = WG ? (vec ? 8 : 32) : (AMODE == 1 ? 4 : 16) + 16;  // VMEM loads per tile
      constexpr int NMF = 48;                                   // MFMAs per tile per wave
#pragma unroll
      for (int i = 0; i < NMF; ++i) {
        if ((i + 1) * NV / NMF != i * NV / NMF) __builtin_amdgcn_sched_group_barrier(0x20, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);  // MFMA
      }
      __syncthreads();  // one buffer: its MFMA reads first
      store_tile(std::integral_constant<int, sb ^ 1>{});
      __syncthreads();
    };
    for (int kt = kb; kt < ke; kt += 2) {
      step(I0{}, kt);
      if (kt + 1 < ke) step(I1{}, kt + 1);
    }
  };
  if constexpr (!WG) {
    if (kt0 < kt1) {
      const int tap = kt0 / p.nbT;
      run(kt0, kt1, tap, kt0 - tap * p.nbT, p.nbT, std::false_type{});
    }
  } else {
    // K classes (host-built): tiles [cstart[c], cstart[c+1]) are (b, j) row-major with
    // ccnt[c] tiles per row at times ct0[c] + 32 j; boundary classes have ccnt = 1.
    for (int c = 0; c < p.ncls; ++c) {
      const int kb = max(kt0, p.cstart[c]);
      const int ke = min(kt1, p.cstart[c + 1]);
      if (kb >= ke) continue;
      const int rel = kb - p.cstart[c];
      const int row = rel / p.ccnt[c];
      const int r0 = (p.Tp == 16 ? 2 : 1) * row, j0 = rel - row * p.ccnt[c];
      // the setup inside each branch: the x4 branch keeps only vB[u][0] live
      if (p.cmask[c] == 0 && p.ta == 1 && p.wvec) {
        wg_class_setup(p.ct0[c], false);
        run(kb, ke, r0, j0, p.ccnt[c], std::true_type{});
      } else {
        wg_class_setup(p.ct0[c], p.cmask[c] != 0);
        run(kb, ke, r0, j0, p.ccnt[c], std::false_type{});
      }
    }
  }

  // ---- epilogue: accumulators -> LDS tile -> row-contiguous stores ----
  float* Cs = lds;  // BM x BN floats: the planes' space
  const int nl = tid & (BN - 1);
  const int n = n0 + nl;
  // the tile's bias values, staged once in LDS (read back as broadcasts: a wave's row is
  // uniform), instead of a dependent global load per stored element
  __shared__ float s_bias[BM];
  const bool use_bias = !WG && !slab && p.splitk <= 1 && p.bias != nullptr;
  if (use_bias && tid < BM) s_bias[tid] = m0 + tid < p.M ? p.bias[m0 + tid] : 0.f;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ml = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int nl2 = wn * 64 + j * 32 + r32;
        Cs[ml * BN + nl2] = acc[i][j][r];
      }
  __syncthreads();
  if (n < p.N) {
    for (int ml = tid >> 7; ml < BM; ml += NTHR / BN) {
      const int m = m0 + ml;
      if (m >= p.M) break;
      const float v = Cs[ml * BN + nl];
      if (slab) {
        slab[ml * BN + nl] = v;
      } else if (p.splitk > 1) {
        p.ws[((long long)split * p.M + m) * p.N + n] = v;
      } else if constexpr (WG) {
        wgrad_store(p, m, n, v);
      } else {
        conv_store_b(p, m, n, v, use_bias ? s_bias[ml] : 0.f);
      }
    }
  }
  __syncthreads();  // Cs aliases the planes the next pass (stream-K) starts writing
}

// ---------------------------------------------------------------------------------------------
// Wide conv/dgrad tile (round 4, MST_GEMM_WIDE=1 A/B): 128 x 256 output tile, 512 threads =
// 8 waves (2 x 4 over 64 x 64 wave tiles), ONE workgroup per CU. The A tile (128 x 32) is loaded
// and split once for 256 columns; the bf16 planes are double-buffered (2 x 72 KB), so iteration
// k runs tile k's MFMAs from one buffer while it splits and stores tile k+1 (loaded one iteration
// earlier) into the other: one workgroup barrier per K tile, and the split/store work sits beside
// the workgroup's own MFMAs instead of relying on a second workgroup on the CU. Threads form two
// 256-thread groups g: group g loads A units 2g, 2g+1 and the B half n0 + 128 g (all 4 units), so
// the per-thread loader is the 128 x 128 kernel's with 6 units instead of 8.
constexpr int BNW = 256, NTHRW = 512;

// Interleave of the split with the MFMAs (sched_group_barrier): MST_W_VPM split VALU per MFMA
// and one LDS store per MST_W_DSE MFMAs, so the 12 plane stores of a K tile land in its first
// 24 MFMA slots. Swept on gemm_micro and the step (profiles/r04/gemm_micro_m11_*, m12_*): one
// store per 4 MFMAs (the first version) 148.5 TF/s for a T = 252 conv fwd, per 2: 156.7-158.8,
// per 1: 157.1-157.4, per 6: 138.8; 2 or 4 VALU per MFMA were no better than 3.
#ifndef MST_W_VPM
#define MST_W_VPM 3
#endif
#ifndef MST_W_DSE
#define MST_W_DSE 2
#endif
constexpr int PLANE_BW = BNW * LDKB;              // bf16 elements per B plane (256 rows)
constexpr int STAGE_BF = 3 * PLANE + 3 * PLANE_BW;  // bf16 elements per stage (72 KB)
constexpr int LDS_W_FLOATS = STAGE_BF;            // two stages = 144 KB; the 128 KB epilogue tile aliases
static_assert(BM * BNW <= LDS_W_FLOATS, "epilogue tile must fit the two stages");

// Split-K slab of a 128 x 256 tile from the LDS tile: one dwordx4 per thread per row, 16 row
// passes with 32-bit offsets (the per-element stores did 64-bit index math for every element:
// the weight-gradient kernels' short-K splits spent more VALU in that epilogue than in their
// main loops, PMC VALU:MFMA 2.3 against 0.33 in the loop).
__device__ __forceinline__ void store_slab4(const GP& p, const float* Cs, int m0, int n0, int split,
                                            int tid) {
  constexpr int Q = BNW / 4, RPP = NTHRW / Q;
  const long long MN = (long long)p.M * p.N;
  const int q = tid & (Q - 1), r0 = tid / Q;
  const int n = n0 + 4 * q;
  const rsrc_t rs = mk_rsrc(p.ws + split * MN, MN);
  const int nrow = p.M - m0 < BM ? p.M - m0 : BM;
#pragma unroll
  for (int i = 0; i < BM / RPP; ++i) {
    const int ml = r0 + RPP * i;
    const f32x4 v = *reinterpret_cast<const f32x4*>(Cs + ml * BNW + 4 * q);
    const uint32_t vo = (ml < nrow && n < p.N) ? (uint32_t)((m0 + ml) * p.N + n) * 4u : OOB;
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)vo, 0, 0);
  }
}

template <int TAPS, int AMODE, bool DUAL>
__device__ __forceinline__ void tile_pass_w(const GP& p, float* lds, int m_t, int n_t, int kt0,
                                            int kt1, int split, int tid) {
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int g = __builtin_amdgcn_readfirstlane(tid >> 8);  // thread group (B half)
  const int t = tid & 255;
  const int wm = (wave >> 1) & 1, wn = wave & 1;
  const int m0 = m_t * BM;
  const int nb0 = n_t * BNW + 128 * g;  // this group's B rows
  auto km_r = [&](int u) __attribute__((always_inline)) { return (t >> 3) + 32 * u; };
  const int km_q = t & 7;
  const int rm_row = t & 127;
  const int kw = __builtin_amdgcn_readfirstlane((tid >> 7) & 1);

  f32x4 ra[2][2], rb[2][4];  // two register stages: 2 A units (u = 2 g + j) and 4 B units
  const rsrc_t rA = mk_rsrc(p.A, p.nA);
  uint32_t rowA[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int u = 2 * g + j;
    const int m = m0 + (AMODE == 2 ? rm_row : km_r(u));
    rowA[j] = m < p.M ? (uint32_t)(m * p.sAm + (AMODE == 2 ? 0 : 4 * km_q * p.sAc)) * 4u : OOB;
  }
  int tinb;
  uint32_t colb0, colb1;
  {
    const int n = nb0 + rm_row;
    const int bb = n / p.Tn;
    const int tt = n - bb * p.Tn;
    tinb = n < p.N ? p.ta * tt + p.tb : -(1 << 29);
    colb0 = (uint32_t)(bb * p.sb0) * 4u;
    colb1 = DUAL ? (uint32_t)(bb * p.sb1) * 4u : 0u;
  }
  auto load_tile = [&](auto S, int tap, int blk) __attribute__((always_inline)) {
    constexpr int st_ = decltype(S)::value;
    const bool s1 = DUAL && blk >= p.nb0;
    const int cb = (s1 ? blk - p.nb0 : blk) * BK;
    const int ci = cb + sel(s1, p.C0, 0);
    const int Cs = sel(s1, p.C1, p.C0);
    const int sA = (ci * p.sAc + tap * p.sAt) * 4;
    if constexpr (AMODE == 1) {
#pragma unroll
      for (int j = 0; j < 2; ++j) ra[st_][j] = ldbs4(rA, rowA[j], sA);
    } else if constexpr (AMODE == 0) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) ra[st_][j][i] = ldbs(rA, rowA[j], sA + i * p.sAc * 4);
    } else {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          ra[st_][j][i] = ldbs(rA, rowA[0], sA + (4 * rm_quad(kw, 2 * g + j) + i) * p.sAc * 4);
    }
    const int tin = tinb + p.tg * tap;
    const int ts = tin + sel(s1, p.off1, p.off0);
    const bool ok = ((unsigned)tin < (unsigned)p.Tv) & ((unsigned)ts < (unsigned)sel(s1, p.T1, p.T0));
    const uint32_t lo = ok ? sel(s1, colb1, colb0) + (uint32_t)ts * 4u : OOB;
    const float* xs = sel(DUAL && s1, p.x1, p.x0);
    const long long ns = sel(DUAL && s1, p.nx1, p.nx0);
    const int scb = sel(s1, p.sc1, p.sc0) * 4;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = cb + 4 * rm_quad(kw, u) + i;
        rb[st_][u][i] = ldbs(mk_rsrc(xs, c < Cs ? ns : 0), lo, c * scb);
      }
  };
  auto store_tile = [&](auto S, int buf) __attribute__((always_inline)) {
    constexpr int st = decltype(S)::value;
    __bf16* Ap = reinterpret_cast<__bf16*>(lds) + buf * STAGE_BF;
    __bf16* Bp = Ap + 3 * PLANE;
    if constexpr (AMODE == 2) {  // this group's A quads 4 kw + 2 g + (0, 1): one pair
      split_store8<PLANE>(Ap, rm_row, 2 * kw + g, ra[st][0], ra[st][1]);
    } else {
#pragma unroll
      for (int j = 0; j < 2; ++j) split_store4<PLANE>(Ap, km_r(2 * g + j), km_q, ra[st][j]);
    }
#pragma unroll
    for (int u = 0; u < 4; u += 2)
      split_store8<PLANE_BW>(Bp, 128 * g + rm_row, 2 * kw + u / 2, rb[st][u], rb[st][u + 1]);
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int r32 = lane & 31;
  const int h = lane >> 5;
  auto mfma_tile = [&](int buf) __attribute__((always_inline)) {
    const __bf16* Ap = reinterpret_cast<const __bf16*>(lds) + buf * STAGE_BF;
    const __bf16* Bp = Ap + 3 * PLANE;
    const int ra0 = wm * 64 + r32, rb0 = 128 * g + wn * 64 + r32;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const Split3 b0 = ld_planes<PLANE_BW>(Bp, rb0, 2 * s + h), b1 = ld_planes<PLANE_BW>(Bp, rb0 + 32, 2 * s + h);
      {
        const Split3 a0 = ld_planes<PLANE>(Ap, ra0, 2 * s + h);
        acc[0][0] = mfma_x6(a0, b0, acc[0][0]);
        acc[0][1] = mfma_x6(a0, b1, acc[0][1]);
      }
      {
        const Split3 a1 = ld_planes<PLANE>(Ap, ra0 + 32, 2 * s + h);
        acc[1][0] = mfma_x6(a1, b0, acc[1][0]);
        acc[1][1] = mfma_x6(a1, b1, acc[1][1]);
      }
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  if (kt0 < kt1) {
    int tap = kt0 / p.nbT, blk = kt0 - tap * p.nbT;
    auto advance = [&]() __attribute__((always_inline)) {
      if (++blk == p.nbT) {
        blk = 0;
        ++tap;
      }
    };
    // tile i (from kt0) lives in register stage i & 1 and LDS buffer i & 1
    load_tile(I0{}, tap, blk);
    advance();
    load_tile(I1{}, tap, blk);
    advance();
    store_tile(I0{}, 0);
    __syncthreads();
    // Tile i's MFMAs from one buffer, the split and store of tile i + 1 into the other, with the
    // split's VALU and LDS writes and the next loads interleaved between the MFMAs
    // (sched_group_barrier). Running the two groups' phases in opposite order instead (one wave
    // per SIMD on MFMAs while the other splits) measured 9 % slower in the step (round 4).
    auto step = [&](auto S) __attribute__((always_inline)) {
      constexpr int sb = decltype(S)::value;  // this tile's stage / buffer
      load_tile(S, tap, blk);                 // tile i + 2 into the stage tile i left
      advance();
      mfma_tile(sb);
      store_tile(std::integral_constant<int, sb ^ 1>{}, sb ^ 1);  // tile i + 1
      constexpr int NV = (AMODE == 1 ? 2 : 8) + 16;                // VMEM loads per tile
#pragma unroll
      for (int i = 0; i < 48; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                // MFMA
        // next-tile loads spread evenly over the 48 MFMAs (in the first NV slots before: T = 252
        // conv fwd 160.7 -> 165.1, dgrad 175.3 -> 180.8 TF/s, T = 15 +6-8 %, step +2.1 %,
        // profiles/r04/gemm_micro_m15_*)
        if ((i + 1) * NV / 48 != i * NV / 48) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, MST_W_VPM, 0);        // VALU (split)
        if (i % MST_W_DSE == MST_W_DSE - 1) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
      }
      __syncthreads();
    };
    for (int kt = kt0; kt < kt1; kt += 2) {
      step(I0{});
      if (kt + 1 < kt1) step(I1{});
    }
  }

  // ---- epilogue: accumulators -> LDS tile (128 x 256) -> row-contiguous stores ----
  float* Cs = lds;
  const int nl = tid & (BNW - 1);
  const int n = n_t * BNW + nl;
  __shared__ float s_bias_w[BM];
  const bool use_bias = p.splitk <= 1 && p.bias != nullptr;
  if (use_bias && tid < BM) s_bias_w[tid] = m0 + tid < p.M ? p.bias[m0 + tid] : 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ml = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int nl2 = 128 * g + wn * 64 + j * 32 + r32;
        Cs[ml * BNW + nl2] = acc[i][j][r];
      }
  __syncthreads();
  if (p.slab4) {
    store_slab4(p, Cs, m_t * BM, n_t * BNW, split, tid);
    return;
  }
  if (n < p.N) {
    for (int ml = tid >> 8; ml < BM; ml += NTHRW / BNW) {
      const int m = m0 + ml;
      if (m >= p.M) break;
      const float v = Cs[ml * BNW + nl];
      if (p.splitk > 1) p.ws[((long long)split * p.M + m) * p.N + n] = v;
      else conv_store_b(p, m, n, v, use_bias ? s_bias_w[ml] : 0.f);
    }
  }
}

template <int TAPS, int AMODE, bool DUAL>
__global__ __launch_bounds__(NTHRW, 1) void gemm_w_kernel(const GP p) {
  __shared__ __attribute__((aligned(16))) float lds[LDS_W_FLOATS];
  const int nx = (p.N + BNW - 1) / BNW, ny = (p.M + BM - 1) / BM;
  const int W = nx * ny * (int)gridDim.z;
  const int t = xcd_order(blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z), W);
  const int split = t / (nx * ny);
  int m_t, n_t;
  tile_of(t - split * nx * ny, nx, ny, m_t, n_t);
  const int kt0 = (int)((long long)split * p.nk / p.splitk);
  const int kt1 = (int)((long long)(split + 1) * p.nk / p.splitk);
  tile_pass_w<TAPS, AMODE, DUAL>(p, lds, m_t, n_t, kt0, kt1, split, threadIdx.x);
}

static int gemm_wide() {  // conv / dgrad on the 128 x 256 kernel; MST_GEMM_WIDE=0: the 128 x 128 one
  static const int v = [] {
    const char* e = getenv("MST_GEMM_WIDE");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return v;
}

static int wg_vec() {
  static const int v = [] {
    const char* e = getenv("MST_WG_VEC");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return v;
}

// ---------------------------------------------------------------------------------------------
// Pre-split operand planes (round 5). The register-split kernels above split every loaded fp32
// element into its three bf16 pieces once per tile pass, i.e. once for every output tile that
// reads it (5.5 VALU per element, three LDS stores per 8 elements: VALU:MFMA 4.5-5.7 in PMC).
// Here a pack kernel splits each operand element ONCE per GEMM into three bf16 planes in HBM,
// laid out as the GEMM reads them ([rows][K], K contiguous, zero padding and every range mask
// baked in), and gemm_p_kernel moves 16-byte pieces of the planes straight into LDS with
// buffer_load ... lds (no VGPRs, no VALU): its main loop is ds_read + MFMA. LDS image, fragment
// reads and MFMA order are the 128 x 256 kernel's (pl_off swizzle: the per-lane source address
// takes the inverse permutation, the destination stays lane-linear).
//
// Weight gradients (K = (b, t), t padded to Tp): A planes = P (dY or X) rows m, B planes = rows
// n = c * taps + tap of X(b, c, a t + beta + g tap) over both concat sources, masked.
struct PackArgs {
  __bf16* out;   // 3 planes of rows x ld bf16, plane stride ps
  long long ps;
  int ld, rows, taps;
  int B, Tk, Tp;
  int a, beta, g, Tv;
  const float* x0;
  long long sb0;
  int sc0, C0, T0, off0;
  const float* x1;
  long long sb1;
  int sc1, T1, off1;
  int two;  // k3 weight gradient in two copies (see build_wgrad_planes): tap 1 in rows [0, C),
            // taps 0 and 2 in rows [C, 2C) (tap 2 read 2 elements further on), zero row 2C
};

// One thread per (channel, 8 consecutive k), grid-stride over channels x ld/8 items (short rows,
// T = 15 .. 63, pack several channels per workgroup), writing them for every tap (rows
// c taps + tap) from one read of the source. Loads are raw buffer loads through one descriptor
// per source; an element outside its ranges (t >= Tk, b >= B, input time outside [0, Tv) or the
// source) gets the OOB offset: hardware zero, no branches.
__device__ __forceinline__ void pack_body(const PackArgs& a, int bid, int nblk) {
  const int q8 = a.ld >> 3;
  const int chans = a.rows / a.taps;
  const rsrc_t r0 = mk_rsrc(a.x0, (long long)(a.B - 1) * a.sb0 + (long long)(a.C0 - 1) * a.sc0 + a.T0);
  const rsrc_t r1 = a.x1 ? mk_rsrc(a.x1, (long long)(a.B - 1) * a.sb1 +
                                             (long long)(chans - a.C0 - 1) * a.sc1 + a.T1)
                         : r0;
  const int total = (chans + a.two) * q8;  // < 2^31: checked by the host (32-bit index math: a
                                           // 64-bit division per item made the pack 30 % slower)
  for (int it = bid * 256 + threadIdx.x; it < total; it += nblk * 256) {
    const int c = it / q8, kq = it - c * q8;
    if (c == chans) {  // the two-copy layout's zero row (what tap 2's shifted reads run into)
      __bf16* o = a.out + (long long)(2 * chans) * a.ld + 8 * kq;
      const bf16x8 z = {};
      *reinterpret_cast<bf16x8*>(o) = z;
      *reinterpret_cast<bf16x8*>(o + a.ps) = z;
      *reinterpret_cast<bf16x8*>(o + 2 * a.ps) = z;
      continue;
    }
    const bool s1 = c >= a.C0;
    const int cs = s1 ? c - a.C0 : c;
    const int Ts = s1 ? a.T1 : a.T0, off = s1 ? a.off1 : a.off0;
    const int k0 = 8 * kq, b = k0 / a.Tp, t0 = k0 - b * a.Tp;
    const int base = b * (int)(s1 ? a.sb1 : a.sb0) + cs * (s1 ? a.sc1 : a.sc0) + off;
    if (a.a == 1 && a.Tv <= a.Tp &&
        (a.taps == 1 ? a.g == 0 && a.beta == 0 : a.g == 1 && a.beta == -1 && a.taps == 3)) {
      // unit-stride rows (k3 convolutions, taps 3; and the P operand, taps 1): branch-free.
      // Each lane loads ITS OWN 8 elements u = t0 .. t0 + 7 with two dwordx4 loads (dword
      // alignment suffices), out-of-range elements zeroed by selects; a k3 tap window
      // u = t0 - 1 + tap + e takes its two halo elements from the neighbouring lanes (the previous
      // / next 8 k: across a batch-row or channel boundary the halo element is out of range anyway,
      // as Tv <= Tp),
      // the wave's first / last lane from two extra masked loads. Each element is split once.
      const bool rowok = b < a.B;
      const int u0 = t0;
      // the 8 own elements, valid where u < Tv and u + off inside the source; the dwordx4 pair is
      // used where it lies inside the source buffer (the descriptor's extent)
      const long long ext = s1 ? (long long)(a.B - 1) * a.sb1 + (long long)(chans - a.C0 - 1) * a.sc1 + a.T1
                               : (long long)(a.B - 1) * a.sb0 + (long long)(a.C0 - 1) * a.sc0 + a.T0;
      const bool vec = base + u0 >= 0 && (long long)base + u0 + 8 <= ext;
      float own[8];
      {
        const uint32_t vo = (uint32_t)(base + u0) * 4u;
        const uint32_t v0 = vec ? vo : OOB, v1 = vec ? vo + 16u : OOB;
        const f32x4 lo = s1 ? ldb4(r1, v0) : ldb4(r0, v0);
        const f32x4 hi = s1 ? ldb4(r1, v1) : ldb4(r0, v1);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          own[e] = lo[e];
          own[e + 4] = hi[e];
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int u = u0 + e;
        const bool ok = rowok && (unsigned)u < (unsigned)a.Tv && (unsigned)(u + off) < (unsigned)Ts;
        if (!vec) {  // the rare lane whose pair would leave the buffer: element by element
          own[e] = s1 ? ldb(r1, ok ? (uint32_t)(base + u) * 4u : OOB) : ldb(r0, ok ? (uint32_t)(base + u) * 4u : OOB);
        }
        own[e] = ok ? own[e] : 0.f;
      }
      const int lane = threadIdx.x & 63;
      const int ntap = a.taps;
      float hl = 0.f, hr = 0.f;  // u = t0 - 1 and u = t0 + 8
      if (ntap == 3) {
        hl = __shfl_up(own[7], 1, 64);
        hr = __shfl_down(own[0], 1, 64);
        // wave edges: the neighbour item belongs to another wave; load the element itself
        const int ul = u0 - 1, ur = u0 + 8;
        const bool okl = lane == 0 && rowok && (unsigned)ul < (unsigned)a.Tv && (unsigned)(ul + off) < (unsigned)Ts;
        const bool okr = lane == 63 && rowok && (unsigned)ur < (unsigned)a.Tv && (unsigned)(ur + off) < (unsigned)Ts;
        const float el = s1 ? ldb(r1, okl ? (uint32_t)(base + ul) * 4u : OOB) : ldb(r0, okl ? (uint32_t)(base + ul) * 4u : OOB);
        const float er = s1 ? ldb(r1, okr ? (uint32_t)(base + ur) * 4u : OOB) : ldb(r0, okr ? (uint32_t)(base + ur) * 4u : OOB);
        // a halo element is valid only inside this row (t0 > 0 / t0 + 8 < Tv) and the source
        const bool vl = rowok && t0 > 0 && (unsigned)(ul + off) < (unsigned)Ts && ul < a.Tv;
        const bool vr = rowok && (unsigned)ur < (unsigned)a.Tv && (unsigned)(ur + off) < (unsigned)Ts;
        hl = lane == 0 ? el : (vl ? hl : 0.f);
        hr = lane == 63 ? er : (vr ? hr : 0.f);
      }
      Bf3 sp[10];
      sp[0] = split1(hl);
#pragma unroll
      for (int e = 0; e < 8; ++e) sp[e + 1] = split1(own[e]);
      sp[9] = split1(hr);
#pragma unroll
      for (int tap = 0; tap < 3; ++tap) {  // unrolled: sp[] stays in registers
        if (tap >= ntap || (a.two && tap == 2)) break;
        bf16x8 hi, mid, lo;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          // time padding; the two-copy layout's tap-0 copy also holds t = Tk (tap 2 reads it
          // two elements on, at t = Tk - 2)
          const bool ok = t0 + e < a.Tk + (a.two && tap == 0);
          // taps 3: window element e + tap (u = t0 - 1 + tap + e); taps 1: own element e
          const Bf3 v = ntap == 3 ? sp[e + tap] : sp[e + 1];
          hi[e] = ok ? v.h : (__bf16)0.f;
          mid[e] = ok ? v.m : (__bf16)0.f;
          lo[e] = ok ? v.l : (__bf16)0.f;
        }
        const int orow = a.two ? (tap == 1 ? c : chans + c) : c * ntap + tap;
        __bf16* o = a.out + (long long)orow * a.ld + k0;
        *reinterpret_cast<bf16x8*>(o) = hi;
        *reinterpret_cast<bf16x8*>(o + a.ps) = mid;
        *reinterpret_cast<bf16x8*>(o + 2 * a.ps) = lo;
      }
      continue;
    }
    for (int tap = 0; tap < a.taps; ++tap) {
      float v[8];
      const int s0 = a.a * t0 + a.beta + a.g * tap;  // input time of element 0
      // interior unit-stride windows: two dwordx4 loads (dword alignment suffices; the tap shift
      // makes most windows 16-byte unaligned); the rest element by element with masks
      const bool interior = a.a == 1 && b < a.B && t0 + 7 < a.Tk && s0 >= 0 && s0 + 7 < a.Tv &&
                            s0 + off >= 0 && s0 + 7 + off < Ts;
      if (interior) {
        const uint32_t vo = (uint32_t)(base + s0) * 4u;
        const f32x4 lo = s1 ? ldb4(r1, vo) : ldb4(r0, vo);
        const f32x4 hi = s1 ? ldb4(r1, vo + 16u) : ldb4(r0, vo + 16u);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = lo[e];
          v[e + 4] = hi[e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int t = t0 + e;
          const int tin = s0 + a.a * e;
          const bool ok = b < a.B && t < a.Tk && (unsigned)tin < (unsigned)a.Tv &&
                          (unsigned)(tin + off) < (unsigned)Ts;
          const uint32_t vo = ok ? (uint32_t)(base + tin) * 4u : OOB;
          v[e] = s1 ? ldb(r1, vo) : ldb(r0, vo);
        }
      }
      bf16x8 hi, mid, lo;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const Bf3 t3 = split1(v[e]);
        hi[e] = t3.h;
        mid[e] = t3.m;
        lo[e] = t3.l;
      }
      __bf16* o = a.out + (long long)(c * a.taps + tap) * a.ld + k0;
      *reinterpret_cast<bf16x8*>(o) = hi;
      *reinterpret_cast<bf16x8*>(o + a.ps) = mid;
      *reinterpret_cast<bf16x8*>(o + 2 * a.ps) = lo;
    }
  }
}

// Both operands' packs of one weight gradient in ONE launch (blocks [0, nba) pack A, the rest B):
// one launch fewer per layer on the weight-gradient stream.
__global__ __launch_bounds__(256) void pack_planes_kernel(const PackArgs a, const PackArgs b, int nba) {
  if ((int)blockIdx.x < nba) pack_body(a, blockIdx.x, nba);
  else pack_body(b, blockIdx.x - nba, gridDim.x - nba);
}

constexpr int STAGE_P = STAGE_BF;  // 72 KB of bf16 per stage: A 3 x [128][32], B 3 x [256][32]

// LDS-DMA piece (buffer_load_dwordx4 ... lds) as inline asm. As a builtin, hipcc inserts
// s_waitcnt vmcnt(0) before the first ds_read after it (the DMA may alias the read), i.e. every K
// tile waited for the NEXT stage's pieces before reading the current one. The asm is invisible to
// that pass; the loop waits for its own pieces (vmcnt(0), then the barrier) before the stage is
// read. M0 is saved and restored inside the statement (as fft.hip's dma_b128).
__device__ __forceinline__ void dma_piece(rsrc_t rs, unsigned lds_addr, uint32_t voff, int soff) {
  unsigned keep;
  asm volatile(
      "s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rs), "s"(lds_addr), "s"(soff)
      : "memory");
}

// Round 6 (tools/micro/gemm_planes.hip, profiles/r06/gemm_planes_micro_stagger.txt): the asm DMA,
// plus two measures for the two waves that share each SIMD (waves w and w + 4 run the same loop
// in lockstep, reaching their fragment reads and the barrier together; MI355X_MICROARCH.md, "two
// waves per SIMD", items 4 and 9):
//  - a STAGGER: waves 4-7 run each K tile's second 16-deep half one barrier late, from fragments
//    read into registers before the barrier (48 VGPRs), so after every barrier one wave per SIMD
//    has MFMAs to issue at once while its partner reads its first fragments;
//  - static priority s_setprio 1 for waves 4-7 (the arbitration losers otherwise).
// The same products are summed in the same order per accumulator, so results are bitwise those of
// the unstaggered loop. Micro: +2-5 % over the builtin-DMA loop on the step's wgrad / conv shapes
// (e.g. 188.6 -> 195.7 TF/s on the L0 audio weight gradient, 172.7 -> 178.9 on L1).
template <bool WG>
__device__ __forceinline__ void tile_pass_p(const GP& p, char* lds, int m_t, int n_t, int kt0,
                                            int kt1, int split, int tid) {
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = m_t * BM, n0 = n_t * BNW;
  const rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)p.pA, (short)0,
                                                      (int)(3 * p.psa * 2), 0x00020000);
  const rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)p.pB, (short)0,
                                                      (int)(3 * p.psb * 2), 0x00020000);
  // this wave's 9 of the stage's 72 one-KB pieces: j = wave + 8 i; j < 24 are A (plane j / 8,
  // rows 16 (j % 8) ..), the rest B (plane (j - 24) / 16, rows 16 ((j - 24) % 16) ..). Lane l
  // fills bytes 16 l of its piece: tile row r0 + l / 4, LDS slot l % 4 = quad q ^ pl_swz(row).
  uint32_t voff[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int j = wave + 8 * i;
    const bool a = j < 24;
    const int jj = a ? j : j - 24;
    const int plane = a ? jj >> 3 : jj >> 4;
    const int r = (a ? jj & 7 : jj & 15) * 16 + (lane >> 2);
    const int q = (lane & 3) ^ pl_swz(r);
    const int row = (a ? m0 : n0) + r;
    const bool in = row < (a ? p.M : p.N);
    // two-copy B planes: row n = 3 c + tap reads copy row c (tap 1) or C + c (taps 0, 2), tap 2
    // two elements (4 bytes: dword-aligned) further along k
    const int c3 = row / 3, tp = row - 3 * c3;
    const int srow = (!a && p.b2) ? (tp == 1 ? c3 : p.bC + c3) : row;
    const int eoff = (!a && p.b2 && tp == 2) ? 2 : 0;
    const long long e = plane * (a ? p.psa : p.psb) + (long long)srow * p.pld + 8 * q + eoff;
    voff[i] = in ? (uint32_t)(e * 2) : OOB;
  }
  const unsigned lds0 = (unsigned)(uintptr_t)lds;  // LDS byte address (low half of the flat one)
  auto issue = [&](int stage, int kt) __attribute__((always_inline)) {
    const int soff = kt * BK * 2;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int j = wave + 8 * i;  // wave-uniform: A or B by a scalar branch
      const unsigned dst = __builtin_amdgcn_readfirstlane(lds0 + (stage * STAGE_P) * 2 + j * 1024);
      if (j < 24) dma_piece(rA, dst, voff[i], soff);
      else dma_piece(rB, dst, voff[i], soff);
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
  const bool late = wave >= 4;  // the second wave on each SIMD
  if (late) __builtin_amdgcn_s_setprio(1);
  if (kt0 < kt1) {
    issue(0, kt0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (!late) {
      for (int kt = kt0; kt < kt1; ++kt) {
        const int st = (kt - kt0) & 1;
        if (kt + 1 < kt1) issue(st ^ 1, kt + 1);
        const __bf16* Ap = reinterpret_cast<const __bf16*>(lds) + st * STAGE_P;
        const __bf16* Bp = Ap + 3 * PLANE;
#pragma unroll
        for (int s2 = 0; s2 < BK / 16; ++s2) {
          const Split3 b0 = ld_planes<PLANE_BW>(Bp, rb0, 2 * s2 + h);
          const Split3 b1 = ld_planes<PLANE_BW>(Bp, rb0 + 32, 2 * s2 + h);
          const Split3 a0 = ld_planes<PLANE>(Ap, ra0, 2 * s2 + h);
          acc[0][0] = mfma_x6(a0, b0, acc[0][0]);
          acc[0][1] = mfma_x6(a0, b1, acc[0][1]);
          const Split3 a1 = ld_planes<PLANE>(Ap, ra0 + 32, 2 * s2 + h);
          acc[1][0] = mfma_x6(a1, b0, acc[1][0]);
          acc[1][1] = mfma_x6(a1, b1, acc[1][1]);
        }
        // the next stage's DMA has landed and every wave is done reading this one
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    } else {
      Split3 pa0, pa1, pb0, pb1;  // the previous K tile's second half, read before the barrier
      for (int kt = kt0; kt < kt1; ++kt) {
        const int st = (kt - kt0) & 1;
        if (kt + 1 < kt1) issue(st ^ 1, kt + 1);
        if (kt > kt0) half(pa0, pa1, pb0, pb1);
        const __bf16* Ap = reinterpret_cast<const __bf16*>(lds) + st * STAGE_P;
        const __bf16* Bp = Ap + 3 * PLANE;
        {
          const Split3 b0 = ld_planes<PLANE_BW>(Bp, rb0, h), b1 = ld_planes<PLANE_BW>(Bp, rb0 + 32, h);
          const Split3 a0 = ld_planes<PLANE>(Ap, ra0, h), a1 = ld_planes<PLANE>(Ap, ra0 + 32, h);
          half(a0, a1, b0, b1);
        }
        pb0 = ld_planes<PLANE_BW>(Bp, rb0, 2 + h);
        pb1 = ld_planes<PLANE_BW>(Bp, rb0 + 32, 2 + h);
        pa0 = ld_planes<PLANE>(Ap, ra0, 2 + h);
        pa1 = ld_planes<PLANE>(Ap, ra0 + 32, 2 + h);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      half(pa0, pa1, pb0, pb1);
    }
  }
  if (late) __builtin_amdgcn_s_setprio(0);
  // epilogue: accumulators -> LDS tile (128 x 256 floats, aliasing the stages) -> rows
  float* Cs = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ml = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int nl = 128 * g + wn * 64 + j * 32 + r32;
        Cs[ml * BNW + nl] = acc[i][j][r];
      }
  __syncthreads();
  if (p.slab4) {
    store_slab4(p, Cs, m0, n0, split, tid);
    return;
  }
  const int nl = tid & (BNW - 1);
  const int n = n0 + nl;
  if (n < p.N) {
    for (int ml = tid >> 8; ml < BM; ml += NTHRW / BNW) {
      const int m = m0 + ml;
      if (m >= p.M) break;
      const float v = Cs[ml * BNW + nl];
      if (p.splitk > 1) p.ws[((long long)split * p.M + m) * p.N + n] = v;
      else if constexpr (WG) wgrad_store(p, m, n, v);
      else conv_store(p, m, n, v);
    }
  }
}

template <bool WG>
__global__ __launch_bounds__(NTHRW, 1) void gemm_p_kernel(const GP p) {
  __shared__ __attribute__((aligned(16))) char lds[LDS_W_FLOATS * 4];
  const int nx = (p.N + BNW - 1) / BNW, ny = (p.M + BM - 1) / BM;
  const int W = nx * ny * (int)gridDim.z;
  const int t = xcd_order(blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z), W);
  const int split = t / (nx * ny);
  int m_t, n_t;
  tile_of(t - split * nx * ny, nx, ny, m_t, n_t);
  const int kt0 = (int)((long long)split * p.nk / p.splitk);
  const int kt1 = (int)((long long)(split + 1) * p.nk / p.splitk);
  tile_pass_p<WG>(p, lds, m_t, n_t, kt0, kt1, split, threadIdx.x);
}

static int wg_two_copy() {  // k3 weight-gradient B planes in two copies; MST_WG_TWO=0: three
  static const int v = [] {
    const char* e = getenv("MST_WG_TWO");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return v;
}

static int wg_planes() {  // weight gradients on pre-split planes; MST_WG_PLANES=0: register split
  static const int v = [] {
    const char* e = getenv("MST_WG_PLANES");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return v;
}

// Schedules. Data-parallel / split-K: one (tile, split) per workgroup, grid (nx, ny, splitk).
// Stream-K: a 1-D grid of G workgroups (one full residency wave); workgroup v runs iterations
// [v L, v L + L) of the flattened (tile, K tile) space, i.e. the tail of one tile, whole tiles,
// then the head of another. A tile covered by one workgroup is finished in place; a tile
// shared by several leaves one partial per workgroup in slab slot 2v (its first tile) or
// 2v + 1 (its last), which sk_fixup_kernel sums in workgroup order. Every workgroup then does
// the same work, so there is no partial last wave.
template <int TAPS, bool WG, int AMODE, bool DUAL>
__global__ __launch_bounds__(NTHR, 2) void gemm_kernel(const GP p) {
  static_assert(6 * PLANE * 2 <= LDS_FLOATS * 4, "bf16 planes must fit the epilogue tile");
  __shared__ __attribute__((aligned(16))) float lds[LDS_FLOATS];
  const int nx = (p.N + BN - 1) / BN, ny = (p.M + BM - 1) / BM;
  if (p.sk_L == 0) {
    const int W = nx * ny * (int)gridDim.z;
    const int t = xcd_order(blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z), W);
    const int split = t / (nx * ny);
    int m_t, n_t;
    tile_of(t - split * nx * ny, nx, ny, m_t, n_t);
    const int kt0 = (int)((long long)split * p.nk / p.splitk);
    const int kt1 = (int)((long long)(split + 1) * p.nk / p.splitk);
    tile_pass<TAPS, WG, AMODE, DUAL>(p, lds, m_t, n_t, kt0, kt1, split, nullptr, threadIdx.x);
    return;
  }
  const int v = xcd_order(blockIdx.x, gridDim.x);
  long long it = (long long)v * p.sk_L;
  const long long it1 = it + p.sk_L < p.sk_I ? it + p.sk_L : p.sk_I;
  int slot = 0;
  while (it < it1) {
    const int t = (int)(it / p.nk);
    const int kt0 = (int)(it - (long long)t * p.nk);
    const int kt1 = it1 - it < (long long)(p.nk - kt0) ? kt0 + (int)(it1 - it) : p.nk;
    int m_t, n_t;
    tile_of(t, nx, ny, m_t, n_t);
    float* slab = (kt0 == 0 && kt1 == p.nk) ? nullptr
                                            : p.ws + (long long)(2 * v + slot) * (BM * BN);
    tile_pass<TAPS, WG, AMODE, DUAL>(p, lds, m_t, n_t, kt0, kt1, 0, slab, threadIdx.x);
    it += kt1 - kt0;
    slot = 1;
  }
}

// Stream-K fixup: one workgroup per (tile, quarter of its rows). A tile finished in place
// (one covering workgroup) is skipped; otherwise the partials of workgroups v0..v1 are summed
// in that order (K order) and stored through the normal epilogue.
template <bool WG>
__global__ __launch_bounds__(256) void sk_fixup_kernel(const GP p) {
  const int t = blockIdx.x;
  const long long L = p.sk_L;
  const int v0 = (int)((long long)t * p.nk / L);
  const int v1 = (int)(((long long)(t + 1) * p.nk - 1) / L);
  if (v0 == v1) return;
  const int nx = (p.N + BN - 1) / BN, ny = (p.M + BM - 1) / BM;
  int m_t, n_t;
  tile_of(t, nx, ny, m_t, n_t);
  const int c4 = (threadIdx.x & 31) * 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int ml = blockIdx.y * 32 + (threadIdx.x >> 5) + 8 * r;
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    for (int v = v0; v <= v1; ++v) {
      const int slot = (int)((long long)v * L / p.nk) == t ? 0 : 1;
      s += *reinterpret_cast<const f32x4*>(p.ws + (long long)(2 * v + slot) * (BM * BN) +
                                           ml * BN + c4);
    }
    const int m = m_t * BM + ml;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (WG) wgrad_store(p, m, n_t * BN + c4 + e, s[e]);
      else conv_store(p, m, n_t * BN + c4 + e, s[e]);
    }
  }
}

template <bool WG>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const GP p) {
  long long total = (long long)p.M * p.N;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    int m = (int)(i / p.N);
    int n = (int)(i - (long long)m * p.N);
    float v = 0.f;
    for (int s = 0; s < p.splitk; ++s) v += p.ws[(long long)s * total + i];
    if constexpr (WG) wgrad_store(p, m, n, v);
    else conv_store(p, m, n, v);
  }
}

// Same reduction, four consecutive elements per thread: float4 slab reads, 32-bit index math
// (host checks M*N % 4 == 0 and M*N < 2^31). Slabs are summed in split order (deterministic,
// identical to the scalar kernel), four slabs' loads in flight at a time.
template <bool WG>
__global__ __launch_bounds__(256) void splitk_reduce4_kernel(const GP p) {
  const int total = p.M * p.N;
  const int q4 = total >> 2;
  const f32x4* ws = reinterpret_cast<const f32x4*>(p.ws);
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < q4; j += gridDim.x * blockDim.x) {
    f32x4 v = ws[j];
    int s = 1;
    for (; s + 3 <= p.splitk; s += 3) {
      const f32x4 a = ws[(long long)s * q4 + j], b = ws[(long long)(s + 1) * q4 + j],
                  c = ws[(long long)(s + 2) * q4 + j];
      v += a;
      v += b;
      v += c;
    }
    for (; s < p.splitk; ++s) v += ws[(long long)s * q4 + j];
    int m = (4 * j) / p.N;
    int n = 4 * j - m * p.N;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};  // bias values loaded ahead of the stores
    if (!WG && p.bias) {
      int mm = m, nn = n;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bv[e] = p.bias[mm < p.M ? mm : p.M - 1];
        if (++nn == p.N) {
          nn = 0;
          ++mm;
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (WG) wgrad_store(p, m, n, v[e]);
      else conv_store_b(p, m, n, v[e], bv[e]);
      if (++n == p.N) {
        n = 0;
        ++m;
      }
    }
  }
}

// The same reduction by rows (N % 4 == 0): grid (ceil(N/4 / 64), ceil(M / 4)), one wave per row m
// and 64 column quads, so m and n need no division; one division per thread for the conv
// epilogue's (b, t), then t steps through the quad. Slabs summed in split order (bitwise the
// kernels above).
template <bool WG>
__global__ __launch_bounds__(256) void splitk_reduce_rows_kernel(const GP p) {
  const int m = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int n = (blockIdx.x * 64 + (threadIdx.x & 63)) * 4;
  if (m >= p.M || n >= p.N) return;
  const long long MN = (long long)p.M * p.N;
  const float* w = p.ws + (long long)m * p.N + n;
  f32x4 v = *reinterpret_cast<const f32x4*>(w);
  for (int s = 1; s < p.splitk; ++s) v += *reinterpret_cast<const f32x4*>(w + s * MN);
  if constexpr (WG) {
#pragma unroll
    for (int e = 0; e < 4; ++e) wgrad_store(p, m, n + e, v[e]);
  } else {
    const float bm = p.bias ? p.bias[m] : 0.f;
    int b = n / p.Tn, t = n - b * p.Tn;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      conv_store_bt(p, m, b, t, v[e], bm);
      if (++t == p.Tn) {
        t = 0;
        ++b;
      }
    }
  }
}

static int reduce_rows() {  // MST_REDUCE_ROWS=0: the 1-D float4 reduce (A/B)
  static const int v = [] {
    const char* e = getenv("MST_REDUCE_ROWS");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return v;
}

template <bool WG>
void launch_reduce(const GP& p, hipStream_t st) {
  const long long total = (long long)p.M * p.N;
  if (reduce_rows() && p.N % 4 == 0 && p.M < 65535 * 4) {
    hipLaunchKernelGGL((splitk_reduce_rows_kernel<WG>), dim3(ceil_div(p.N / 4, 64), ceil_div(p.M, 4)),
                       dim3(256), 0, st, p);
  } else if (total % 4 == 0 && total < (1ll << 31)) {
    int blocks = (int)((total / 4 + 255) / 256);
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL((splitk_reduce4_kernel<WG>), dim3(blocks), dim3(256), 0, st, p);
  } else {
    int blocks = (int)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL((splitk_reduce_kernel<WG>), dim3(blocks), dim3(256), 0, st, p);
  }
}

// Split-K from a wave-quantisation cost model. 256 CUs x occ resident workgroups = the slots;
// a workgroup's time is ~ (its K tiles) x tau. At occ = 2 a trailing partial wave of <= 256
// workgroups runs one workgroup per CU (no MFMA-pipe sharing) and costs ~0.55 of a full wave;
// at occ = 1 (the 128 x 256 kernels) a lone workgroup runs no faster than in a full wave, so a
// partial wave "should" cost a whole one, but charging it 1.0 (more splits) ran the training step
// 0.8-1.6 % SLOWER (36.65-36.82 vs 37.10-37.24 ms, two same-box alternations,
// profiles/r05/ab_step_w_partial.jsonl; the serialised GEMM leg itself ran faster, 159 -> 167
// TF/s for conv/dgrad): beside the side-stream weight gradients the extra slab traffic and reduce
// launches cost more than the quantisation they remove. MST_W_PARTIAL keeps 0.55, the measured
// winner. Split-K adds a slab round trip (s + 2 passes over M x N floats) plus a launch.
#ifndef MST_W_PARTIAL
#define MST_W_PARTIAL 0.55
#endif
int choose_splitk(int M, int N, int nk, int req, int occ, int bn = BN) {
  if (req > 0) return req < nk ? req : (nk > 0 ? nk : 1);
  const long long tiles = (long long)ceil_div(M, BM) * ceil_div(N, bn);
  static const double tau_env = [] {  // dev override for tuning (MST_SPLITK_TAU seconds)
    const char* e = getenv("MST_SPLITK_TAU");
    return e ? atof(e) : 0.0;
  }();
  const double slots = 256.0 * occ;
  const double tau = tau_env > 0 ? tau_env : 3.4e-6;  // s per 32-deep K tile of one workgroup
  static const double bw = [] {  // slab round-trip bandwidth (MST_SPLITK_BW bytes/s, tuning)
    const char* e = getenv("MST_SPLITK_BW");
    return e ? atof(e) : 8e12;  // 5e12 -> 8e12: 50.5 -> 50.3 ms/step (sweep 2e12-2e13)
  }();
  auto waves = [&](long long n) {
    long long full = n / (long long)slots, rem = n % (long long)slots;
    return (double)full + (rem == 0 ? 0.0 : (rem <= slots / 2 ? (occ == 1 ? MST_W_PARTIAL : 0.55) : 1.0));
  };
  int best = 1;
  double best_t = waves(tiles) * nk * tau;
  const int maxs = nk / 4 < 32 ? nk / 4 : 32;  // at least four K tiles per split
  for (int s = 2; s <= maxs; ++s) {
    const double t = waves(tiles * s) * ceil_div(nk, s) * tau +
                     (double)M * N * 4.0 * (s + 2) / bw + 4e-6;
    if (t < best_t * 0.97) {
      best_t = t;
      best = s;
    }
  }
  return best;
}

// Stream-K: G workgroups = one residency wave (256 CUs x 2), each ceil(I / G) iterations.
constexpr int SK_G = 512;

// Schedule of one GEMM: req > 0 forces that split-K, req == -1 forces stream-K over SK_G
// workgroups, req < -1 stream-K over -req workgroups (tests), req == 0 uses the split-K cost
// model (MST_GEMM_SCHED=sk selects stream-K for A/B runs). Stream-K is not chosen
// automatically: over the training step it was within noise of split-K in time and raised the
// GEMMs' HBM-side traffic from 254 to 322 MB per launch (profiles/r01/gemm_traffic_m14_*.json):
// a workgroup walking several tiles in sequence shares fewer panels through L2 with the
// workgroups running beside it than one tile per workgroup does.
void choose_sched(GP& p, int req) {
  p.sk_L = p.sk_I = 0;
  const long long tiles = (long long)ceil_div(p.M, BM) * ceil_div(p.N, BN);
  int G = 0;
  if (req < 0) {
    G = req == -1 ? SK_G : -req;
  } else if (req == 0) {
    static const bool sk = [] {
      const char* e = getenv("MST_GEMM_SCHED");
      return e && e[0] == 's';
    }();
    if (sk) G = SK_G;
  }
  if (G > 0) {
    p.wide = 0;
    p.splitk = 1;
    p.sk_I = tiles * p.nk;
    p.sk_L = (p.sk_I + G - 1) / G;
  } else {
    p.splitk = p.wide ? choose_splitk(p.M, p.N, p.nk, req, 1, BNW) : choose_splitk(p.M, p.N, p.nk, req, 2);
  }
}

bool slab4_ok(int M, int N, int splitk) {  // MST_SLAB4=0: per-element slab stores (A/B)
  static const int env = [] {
    const char* e = getenv("MST_SLAB4");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return env && splitk > 1 && N % 4 == 0 && (long long)M * N < (1ll << 29);
}

size_t sched_ws_bytes(const GP& p) {
  if (p.sk_L > 0) {  // two partial-tile slots per workgroup of the launched grid
    const long long G = (p.sk_I + p.sk_L - 1) / p.sk_L;
    return p.sk_L % p.nk ? (size_t)(2 * G) * BM * BN * sizeof(float) : 0;
  }
  if (p.splitk <= 1) return 0;
  return (size_t)p.splitk * p.M * p.N * sizeof(float);
}

// Falls back to a single K pass (data-parallel) when the caller's workspace is too small.
void bind_ws(GP& p, float* ws, size_t ws_bytes) {
  const size_t need = sched_ws_bytes(p);
  if (need > 0 && (!ws || ws_bytes < need)) {
    p.sk_L = p.sk_I = 0;
    p.splitk = 1;
  }
  p.ws = ws;
  p.slab4 = p.wide && p.sk_L == 0 && slab4_ok(p.M, p.N, p.splitk);
}

template <bool WG>
int launch(const GP& p, hipStream_t st, int taps) {
  dim3 grid(ceil_div(p.N, BN), ceil_div(p.M, BM), p.splitk);
  if (p.sk_L > 0) grid = dim3((unsigned)((p.sk_I + p.sk_L - 1) / p.sk_L), 1, 1);
  dim3 block(NTHR);
  const bool wide = !WG && p.wide && p.sk_L == 0;
  const dim3 wgrid(ceil_div(p.N, BNW), ceil_div(p.M, BM), p.splitk), wblock(NTHRW);
  // (wide implies !WG: the weight-gradient instantiations never reference gemm_w_kernel)
#define MST_GEMM_LAUNCH(TP, AM)                                                      \
  if (wide) {                                                                        \
    if constexpr (!WG) {                                                             \
      if (p.dual) hipLaunchKernelGGL((gemm_w_kernel<TP, AM, true>), wgrid, wblock, 0, st, p); \
      else hipLaunchKernelGGL((gemm_w_kernel<TP, AM, false>), wgrid, wblock, 0, st, p); \
    }                                                                                \
  } else if (!WG && p.dual)                                                          \
    hipLaunchKernelGGL((gemm_kernel<TP, WG, AM, !WG>), grid, block, 0, st, p);       \
  else                                                                               \
    hipLaunchKernelGGL((gemm_kernel<TP, WG, AM, false>), grid, block, 0, st, p);
#define MST_GEMM_CASE(TP)                                                            \
  case TP:                                                                           \
    if (WG || p.a_mode == 0) {                                                       \
      MST_GEMM_LAUNCH(TP, 0)                                                         \
    } else if (p.a_mode == 1) {                                                      \
      MST_GEMM_LAUNCH(TP, (WG ? 0 : 1))                                              \
    } else {                                                                         \
      MST_GEMM_LAUNCH(TP, (WG ? 0 : 2))                                              \
    }                                                                                \
    break;
  switch (taps) {
    MST_GEMM_CASE(1)
    MST_GEMM_CASE(2)
    MST_GEMM_CASE(3)
    MST_GEMM_CASE(4)
    MST_GEMM_CASE(6)
    default: return MST_EINVAL;
  }
#undef MST_GEMM_CASE
#undef MST_GEMM_LAUNCH
  MST_CHECK_LAUNCH();
  if (p.sk_L > 0 && p.sk_L % p.nk) {
    dim3 fg((unsigned)(p.sk_I / p.nk), BM / 32, 1);
    hipLaunchKernelGGL((sk_fixup_kernel<WG>), fg, dim3(256), 0, st, p);
    MST_CHECK_LAUNCH();
  }
  if (p.splitk > 1) {
    launch_reduce<WG>(p, st);
    MST_CHECK_LAUNCH();
  }
  return MST_OK;
}

bool taps_ok(int t) { return t == 1 || t == 2 || t == 3 || t == 4 || t == 6; }

void fill_src(GP& p, const mst_src* s, int Ctot) {
  p.x0 = s[0].p;
  p.sb0 = s[0].sb;
  p.sc0 = s[0].sc;
  p.C0 = s[0].C;
  p.T0 = s[0].T;
  p.off0 = s[0].off;
  p.x1 = s[1].C > 0 ? s[1].p : nullptr;
  p.dual = s[1].C > 0;
  p.sb1 = s[1].sb;
  p.sc1 = s[1].sc;
  p.T1 = s[1].T;
  p.off1 = s[1].off;
  p.C1 = s[1].C;
  if (s[1].C <= 0) p.C0 = Ctot;  // single source covers all channels
}

// Elements reachable through each source descriptor; every buffer must stay below the 2 GB
// that the 32-bit buffer offsets (and the OOB sentinel) can address.
int src_extent(GP& p, int B) {
  p.nx0 = (long long)(B - 1) * p.sb0 + (long long)(p.C0 - 1) * p.sc0 + p.T0;
  p.nx1 = p.dual ? (long long)(B - 1) * p.sb1 + (long long)(p.C1 - 1) * p.sc1 + p.T1 : 0;
  MST_REQUIRE(p.sb0 >= 0 && p.sc0 >= 0 && p.sb1 >= 0 && p.sc1 >= 0);
  MST_REQUIRE(p.nx0 * 4 < (long long)OOB && p.nx1 * 4 < (long long)OOB);
  return MST_OK;
}

int build_conv(const mst_conv_desc* d, GP& p) {
  MST_REQUIRE(d && d->A && d->src[0].p && d->dst[0].p);
  MST_REQUIRE(d->B > 0 && d->M > 0 && d->Tn > 0 && d->Ctot > 0 && taps_ok(d->taps));
  MST_REQUIRE(d->src[0].C + (d->src[1].C > 0 ? d->src[1].C : 0) == d->Ctot);
  MST_REQUIRE(d->dst[0].C + (d->dst[1].C > 0 ? d->dst[1].C : 0) == d->M);
  MST_REQUIRE(d->dst[1].C <= 0 || d->dst[1].p);
  MST_REQUIRE(d->drop_p >= 0.f && d->drop_p < 1.f);
  p = GP{};
  p.M = d->M;
  p.N = d->B * d->Tn;
  p.A = d->A;
  p.sAm = d->sAm;
  p.sAc = d->sAc;
  p.sAt = d->sAt;
  fill_src(p, d->src, d->Ctot);
  // tap-major K with each source's channels padded to whole BK tiles
  p.nb0 = ceil_div(p.C0, BK);
  p.nbT = p.nb0 + (p.dual ? ceil_div(p.C1, BK) : 0);
  p.nk = p.nbT * d->taps;
  p.K = p.nk * BK;
  const bool kvec = d->sAc == 1 && (d->sAm % 4) == 0 && (d->taps == 1 || (d->sAt % 4) == 0) &&
                    (p.C0 % 4) == 0 && ((uintptr_t)d->A % 16) == 0;
  const long long am = d->sAm < 0 ? -d->sAm : d->sAm;
  p.a_mode = kvec ? 1 : (am <= 8 ? 2 : 0);
  p.nA = (long long)(p.M - 1) * d->sAm + (long long)(d->Ctot - 1) * d->sAc +
         (long long)(d->taps - 1) * d->sAt + 1;
  MST_REQUIRE(d->sAm >= 0 && d->sAc >= 0 && d->sAt >= 0);
  MST_REQUIRE(src_extent(p, d->B) == MST_OK && p.nA * 4 < (long long)OOB);
  p.Tv = d->Tv;
  p.ta = d->a;
  p.tb = d->beta;
  p.tg = d->g;
  p.Tn = d->Tn;
  p.ostride = d->ostride;
  p.ophase = d->ophase;
  p.y0 = d->dst[0].p;
  p.yb0 = d->dst[0].sb;
  p.yc0 = d->dst[0].sc;
  p.M0 = d->dst[0].C;
  p.yT0 = d->dst[0].T;
  p.yoff0 = d->dst[0].off;
  p.gt0 = d->dst[0].gate;
  p.gs0 = d->dst[0].gate_scale;
  p.y1 = d->dst[1].C > 0 ? d->dst[1].p : nullptr;
  p.yb1 = d->dst[1].sb;
  p.yc1 = d->dst[1].sc;
  p.yT1 = d->dst[1].T;
  p.yoff1 = d->dst[1].off;
  p.gt1 = d->dst[1].gate;
  p.gs1 = d->dst[1].gate_scale;
  p.alpha = d->alpha;
  p.bias = d->bias;
  p.act = d->act;
  p.drop_p = d->drop_p;
  p.seed = d->seed;
  p.seed_dev = reinterpret_cast<const unsigned long long*>(d->seed_dev);
  p.wide = gemm_wide();
  choose_sched(p, d->splitk);
  return MST_OK;
}

// Weight-gradient GEMM over ONE input source (a virtual concat is split into one launch per
// source by the caller): columns [0, C*taps) of `out` for that source's channels.
int build_wgrad(const mst_wgrad_desc* d, const mst_src& src, float* out, GP& p) {
  MST_REQUIRE(d && d->P && src.p && out);
  MST_REQUIRE(d->B > 0 && d->M > 0 && d->Tk > 0 && src.C > 0 && taps_ok(d->taps));
  MST_REQUIRE(d->g >= 0 && d->a >= 1);
  p = GP{};
  p.M = d->M;
  p.N = src.C * d->taps;
  // time axis padded to Tp: 16 for short rows, else a multiple of BK (a tile = one batch row)
  p.Tp = d->Tk <= 16 ? 16 : ceil_div(d->Tk, BK) * BK;
  p.P = d->P;
  p.sPb = d->sPb;
  p.sPc = d->sPc;
  p.Tk = d->Tk;
  mst_src one[2] = {src, mst_src{}};
  fill_src(p, one, src.C);
  p.nP = (long long)(d->B - 1) * d->sPb + (long long)(d->M - 1) * d->sPc + d->Tk;
  MST_REQUIRE(src_extent(p, d->B) == MST_OK && p.nP * 4 < (long long)OOB);
  MST_REQUIRE(p.sPb * 2 < (long long)OOB / 4);
  p.Tv = d->Tv;
  p.ta = d->a;
  p.tb = d->beta;
  p.tg = d->g;
  // valid input times: 0 <= tin < Tv and 0 <= tin + off < T
  const int lo = src.off < 0 ? -src.off : 0;
  const int hi = d->Tv < src.T - src.off ? d->Tv : src.T - src.off;
  p.lo = lo;
  p.span = hi > lo ? hi - lo : 0;
  // K classes: per time tile j (t0 = 32 j) of a batch row, "interior" when every element of
  // every row is in range; consecutive interior tiles share one unmasked class, every other
  // tile is a masked class of its own (ranges are monotone in t0, so there are few).
  const int rows = p.Tp == 16 ? ceil_div(d->B, 2) : d->B;
  const int nj = p.Tp == 16 ? 1 : p.Tp / BK;
  p.ncls = 0;
  int start = 0;
  for (int j = 0; j < nj;) {
    const int t0 = BK * j;
    auto interior = [&](int t) {
      const int st = d->a * t + d->beta;
      return t + BK <= d->Tk && st >= p.lo && st + d->a * (BK - 1) + d->g * (d->taps - 1) < p.lo + p.span;
    };
    int cnt = 1;
    const bool in = interior(t0);
    if (in)
      while (j + cnt < nj && interior(BK * (j + cnt))) ++cnt;
    MST_REQUIRE(p.ncls < MAXCLS);
    p.cstart[p.ncls] = start;
    p.ct0[p.ncls] = t0;
    p.ccnt[p.ncls] = cnt;
    p.cmask[p.ncls] = in ? 0 : 1;
    ++p.ncls;
    start += rows * cnt;
    j += cnt;
  }
  p.cstart[p.ncls] = start;
  p.nk = start;
  p.K = p.nk * BK;
  p.out = out;
  p.ldo = d->ldo;
  p.taps = d->taps;
  if (d->ldc == 0 && d->ldt == 0) {
    p.ldc = d->taps;
    p.ldt = 1;
  } else {
    p.ldc = d->ldc;
    p.ldt = d->ldt;
  }
  p.ocustom = !(p.ldc == d->taps && p.ldt == 1);
  p.inv_taps = 1.0f / (float)d->taps;
  MST_REQUIRE(p.N < (1 << 22));
  p.scale = d->scale;
  p.accumulate = d->accumulate;
  p.wvec = wg_vec();
  choose_sched(p, d->splitk);
  return MST_OK;
}

// Weight gradient on pre-split planes: ONE GEMM over both concat sources (columns n = c taps + tap
// of the concatenated channels, which is where the per-source launches' outputs sit too).
// Workspace: [split-K slabs][A planes][B planes], 256-byte aligned pieces.
struct PlanesWG {
  GP p;
  PackArgs pa, pb;
  size_t slab_bytes, a_bytes, b_bytes;
};

static size_t round256(size_t x) { return (x + 255) / 256 * 256; }

int build_wgrad_planes(const mst_wgrad_desc* d, PlanesWG& w) {
  MST_REQUIRE(d && d->P && d->src[0].p && d->out);
  MST_REQUIRE(d->B > 0 && d->M > 0 && d->Tk > 0 && d->Ctot > 0 && d->src[0].C > 0 && taps_ok(d->taps));
  MST_REQUIRE(d->g >= 0 && d->a >= 1);
  MST_REQUIRE(d->src[0].C + (d->src[1].C > 0 ? d->src[1].C : 0) == d->Ctot);
  MST_REQUIRE(d->src[1].C <= 0 || d->src[1].p);
  GP& p = w.p;
  p = GP{};
  p.M = d->M;
  p.N = d->Ctot * d->taps;
  MST_REQUIRE(p.N < (1 << 22));
  const int Tp = d->Tk <= 16 ? 16 : ceil_div(d->Tk, BK) * BK;
  const int Bp = Tp == 16 ? (d->B + 1) / 2 * 2 : d->B;  // K a multiple of BK
  const long long Kp = (long long)Bp * Tp;
  MST_REQUIRE(Kp < (1 << 30));
  p.pld = (int)Kp;
  p.K = (int)Kp;
  p.nk = (int)(Kp / BK);
  p.psa = (long long)p.M * Kp;
  // k3 convolutions' weight gradient (unit stride, the pack's fast path) with at least one
  // padding step after each batch row (Tp > Tk): the three tap-shifted copies of X become two,
  // tap 1 and tap 0 (= tap 2 read two elements further: 4 bytes, which LDS-DMA takes), 12 instead
  // of 18 bytes per element written by the pack and fetched by the GEMM. A shifted read that runs
  // past a batch row lands on the next row's leading zero (valid t) or meets dY = 0 (padding t),
  // and past a channel's last row on the next channel's leading zero or the zero row 2C.
  p.b2 = wg_two_copy() && d->taps == 3 && d->a == 1 && d->g == 1 && d->beta == -1 && d->Tv <= Tp &&
         Tp > d->Tk;
  p.bC = d->Ctot;
  p.psb = p.b2 ? (long long)(2 * d->Ctot + 1) * Kp : (long long)p.N * Kp;
  // the plane descriptors address 3 planes with 32-bit byte offsets
  MST_REQUIRE(6 * p.psa < (long long)OOB && 6 * p.psb < (long long)OOB);
  p.out = d->out;
  p.ldo = d->ldo;
  p.taps = d->taps;
  if (d->ldc == 0 && d->ldt == 0) {
    p.ldc = d->taps;
    p.ldt = 1;
  } else {
    p.ldc = d->ldc;
    p.ldt = d->ldt;
  }
  p.ocustom = !(p.ldc == d->taps && p.ldt == 1);
  p.inv_taps = 1.0f / (float)d->taps;
  p.scale = d->scale;
  p.accumulate = d->accumulate;
  p.splitk = choose_splitk(p.M, p.N, p.nk, d->splitk > 0 ? d->splitk : 0, 1, BNW);
  PackArgs& a = w.pa;
  a = PackArgs{};
  a.ps = p.psa;
  a.ld = (int)Kp;
  a.rows = p.M;
  a.taps = 1;
  a.B = d->B;
  a.Tk = d->Tk;
  a.Tp = Tp;
  a.a = 1;
  a.Tv = d->Tk;
  a.x0 = d->P;
  a.sb0 = d->sPb;
  a.sc0 = d->sPc;
  a.C0 = p.M;
  a.T0 = d->Tk;
  PackArgs& b = w.pb;
  b = a;
  b.ps = p.psb;
  b.two = p.b2;
  b.rows = p.N;
  b.taps = d->taps;
  b.a = d->a;
  b.beta = d->beta;
  b.g = d->g;
  b.Tv = d->Tv;
  b.x0 = d->src[0].p;
  b.sb0 = d->src[0].sb;
  b.sc0 = d->src[0].sc;
  b.C0 = d->src[1].C > 0 ? d->src[0].C : d->Ctot;
  b.T0 = d->src[0].T;
  b.off0 = d->src[0].off;
  if (d->src[1].C > 0) {
    b.x1 = d->src[1].p;
    b.sb1 = d->src[1].sb;
    b.sc1 = d->src[1].sc;
    b.T1 = d->src[1].T;
    b.off1 = d->src[1].off;
  }
  MST_REQUIRE((long long)p.N * (Kp / 8) < (1ll << 31) && (long long)p.M * (Kp / 8) < (1ll << 31));
  for (const PackArgs* q : {&a, &b}) {  // 32-bit byte offsets through each source's descriptor
    const int C1 = q->rows / q->taps - q->C0;
    MST_REQUIRE((long long)(q->B - 1) * q->sb0 + (long long)(q->C0 - 1) * q->sc0 + q->T0 < (1ll << 29));
    MST_REQUIRE(!q->x1 || (long long)(q->B - 1) * q->sb1 + (long long)(C1 - 1) * q->sc1 + q->T1 < (1ll << 29));
  }
  w.slab_bytes = p.splitk > 1 ? round256((size_t)p.splitk * p.M * p.N * sizeof(float)) : 0;
  w.a_bytes = round256((size_t)(3 * p.psa) * 2);
  w.b_bytes = round256((size_t)(3 * p.psb) * 2);
  p.slab4 = slab4_ok(p.M, p.N, p.splitk) ? 1 : 0;
  return MST_OK;
}

static unsigned pack_blocks(const PackArgs& a) {
  const long long items = (long long)(a.rows / a.taps + a.two) * (a.ld >> 3);
  long long blocks = (items + 255) / 256;
  return (unsigned)(blocks > 8192 ? 8192 : blocks);
}

int launch_pack2(const PackArgs& a, const PackArgs& b, hipStream_t st) {
  const unsigned na = pack_blocks(a), nb = pack_blocks(b);
  hipLaunchKernelGGL(pack_planes_kernel, dim3(na + nb), dim3(256), 0, st, a, b, (int)na);
  MST_CHECK_LAUNCH();
  return MST_OK;
}

int run_wgrad_planes(PlanesWG& w, float* ws, hipStream_t st) {
  GP& p = w.p;
  char* base = reinterpret_cast<char*>(ws);
  p.ws = ws;
  w.pa.out = reinterpret_cast<__bf16*>(base + w.slab_bytes);
  w.pb.out = reinterpret_cast<__bf16*>(base + w.slab_bytes + w.a_bytes);
  p.pA = w.pa.out;
  p.pB = w.pb.out;
  int rc = launch_pack2(w.pa, w.pb, st);
  if (rc) return rc;
  dim3 grid(ceil_div(p.N, BNW), ceil_div(p.M, BM), p.splitk);
  hipLaunchKernelGGL((gemm_p_kernel<true>), grid, dim3(NTHRW), 0, st, p);
  MST_CHECK_LAUNCH();
  if (p.splitk > 1) {
    launch_reduce<true>(p, st);
    MST_CHECK_LAUNCH();
  }
  return MST_OK;
}

// the planes path serves auto and split-K schedules (stream-K requests take the register path)
bool use_wgrad_planes(const mst_wgrad_desc* d, PlanesWG& w) {
  return d && d->splitk >= 0 && wg_planes() && build_wgrad_planes(d, w) == MST_OK;
}

int wgrad_sources(const mst_wgrad_desc* d, mst_src* srcs, float** outs) {
  MST_REQUIRE(d && d->src[0].C + (d->src[1].C > 0 ? d->src[1].C : 0) == d->Ctot);
  srcs[0] = d->src[0];
  outs[0] = d->out;
  if (d->src[1].C <= 0) return 1;
  srcs[1] = d->src[1];
  const long long ldc = d->ldc == 0 && d->ldt == 0 ? d->taps : d->ldc;
  outs[1] = d->out + (long long)d->src[0].C * ldc;
  return 2;
}

}  // namespace

extern "C" {

int mst_gemm_products(void) { return 6; }

size_t mst_conv_fwd_workspace_size(const mst_conv_desc* d) {
  GP p;
  if (build_conv(d, p) != MST_OK) return 0;
  return sched_ws_bytes(p);
}

int mst_conv_fwd_f32(const mst_conv_desc* d, float* ws, size_t ws_bytes, void* stream) {
  GP p;
  int rc = build_conv(d, p);
  if (rc) return rc;
  bind_ws(p, ws, ws_bytes);
  return launch<false>(p, (hipStream_t)stream, d->taps);
}

size_t mst_wgrad_workspace_size(const mst_wgrad_desc* d) {
  mst_src srcs[2];
  float* outs[2];
  if (!d) return 0;
  PlanesWG w;
  if (use_wgrad_planes(d, w)) return w.slab_bytes + w.a_bytes + w.b_bytes;
  const int ns = wgrad_sources(d, srcs, outs);
  if (ns < 1) return 0;
  size_t need = 0;
  for (int i = 0; i < ns; ++i) {
    GP p;
    if (build_wgrad(d, srcs[i], outs[i], p) != MST_OK) return 0;
    const size_t w = sched_ws_bytes(p);
    need = w > need ? w : need;
  }
  return need;
}

int mst_conv_wgrad_f32(const mst_wgrad_desc* d, float* ws, size_t ws_bytes, void* stream) {
  mst_src srcs[2];
  float* outs[2];
  if (!d) return MST_EINVAL;
  {
    PlanesWG w;
    if (use_wgrad_planes(d, w) && ws && ws_bytes >= w.slab_bytes + w.a_bytes + w.b_bytes &&
        ((uintptr_t)ws & 255) == 0)
      return run_wgrad_planes(w, ws, (hipStream_t)stream);
  }
  const int ns = wgrad_sources(d, srcs, outs);
  if (ns < 1) return MST_EINVAL;
  GP ps[2];
  for (int i = 0; i < ns; ++i) {  // validate every launch before enqueueing any
    int rc = build_wgrad(d, srcs[i], outs[i], ps[i]);
    if (rc) return rc;
  }
  for (int i = 0; i < ns; ++i) {
    GP& p = ps[i];
    bind_ws(p, ws, ws_bytes);
    int rc = launch<true>(p, (hipStream_t)stream, d->taps);
    if (rc) return rc;
  }
  return MST_OK;
}

}  // extern "C"
