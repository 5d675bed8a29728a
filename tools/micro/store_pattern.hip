// Store-pattern microbenchmark (dev tool): writes a (B, F, T) = (256, 1025, 252) fp32 tensor
// (the config-2 STFT output, 264.5 MB) with the access patterns an STFT kernel can produce.
// A workgroup writes RUN consecutive frames of every bin row (RUN*4-byte runs).
//   group 0: workgroup g = (clip, block of RUN frames) in row-major order (g % 8 = XCD label
//            cycles through the blocks of one clip)
//   group 1: the blocks of one clip are dispatched on one XCD (g % 8 fixed per clip)
//   nt:      nontemporal stores
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int B = 256, F = 1025, T = 252;

__global__ __launch_bounds__(512) void contiguous(float4* out, long long n4) {
  for (long long i = blockIdx.x * 512ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 512)
    out[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

template <int RUN, bool NT>
__global__ __launch_bounds__(512) void runs(float* out, int group) {
  const int nblk = (T + RUN - 1) / RUN;
  const int g = blockIdx.x;
  int b, blk;
  if (!group) {
    b = g / nblk;
    blk = g % nblk;
  } else {
    b = (g / (8 * nblk)) * 8 + (g % 8);
    blk = (g / 8) % nblk;
  }
  if (b >= B) return;
  float* ob = out + (long long)b * F * T;
  const int f0 = blk * RUN;
  const int nv = RUN / 4;
  for (int e = threadIdx.x; e < F * nv; e += 512) {
    const int k = e / nv, q = e % nv;
    const int f = f0 + 4 * q;
    float* o = ob + (long long)k * T + f;
    if (f + 3 < T) {
      typedef float f4 __attribute__((ext_vector_type(4)));
      f4 v = {(float)k, (float)f, 1.f, 2.f};
      if (NT) __builtin_nontemporal_store(v, reinterpret_cast<f4*>(o));
      else *reinterpret_cast<f4*>(o) = v;
    } else {
      for (int w = 0; w < 4 && f + w < T; ++w) o[w] = 1.f;
    }
  }
}

// Wave-autonomous pattern (no LDS staging): each wave of a W-wave workgroup owns 4 consecutive
// frames and stores, per lane, one float4 (its 4 frames) for each of the 16 bins it holds
// (k = l + 64 j and 1024 - l - 64 j, as the STFT's register layout), plus bin 512 / 1024 from
// lane 0; the W waves cover 4 W consecutive frames, the clip's blocks stay on one XCD.
template <int W>
__global__ __launch_bounds__(64 * W) void wave4(float* out) {
  const int FR = 4 * W;
  const int nblk = (T + FR - 1) / FR;
  const int g = blockIdx.x;
  const int b = (g / (8 * nblk)) * 8 + (g % 8);
  const int blk = (g / 8) % nblk;
  if (b >= B) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int f = blk * FR + 4 * wave;
  if (f + 3 >= T) return;
  float* ob = out + (long long)b * F * T + f;
  typedef float f4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k0 = lane + 64 * j, k1 = 1024 - lane - 64 * j;
    *reinterpret_cast<f4*>(ob + (long long)k0 * T) = f4{(float)k0, 1.f, 2.f, 3.f};
    if (k1 != k0 && k1 < 1024 && lane + j > 0)
      *reinterpret_cast<f4*>(ob + (long long)k1 * T) = f4{(float)k1, 1.f, 2.f, 3.f};
  }
  if (lane == 0) {
    *reinterpret_cast<f4*>(ob + 512ll * T) = f4{512.f, 1.f, 2.f, 3.f};
    *reinterpret_cast<f4*>(ob + 1024ll * T) = f4{1024.f, 1.f, 2.f, 3.f};
  }
}

int main() {
  float* d;
  const size_t n = (size_t)B * F * T;
  (void)hipMalloc(&d, n * 4);
  hipEvent_t s, e;
  (void)hipEventCreate(&s);
  (void)hipEventCreate(&e);
  auto time = [&](const char* name, auto launch) {
    launch();
    (void)hipEventRecord(s);
    for (int i = 0; i < 20; ++i) launch();
    (void)hipEventRecord(e);
    (void)hipEventSynchronize(e);
    float ms;
    (void)hipEventElapsedTime(&ms, s, e);
    ms /= 20;
    printf("%-28s %.4f ms  %.1f GB/s\n", name, ms, n * 4 / (ms * 1e-3) / 1e9);
  };
  time("contiguous", [&] { contiguous<<<4096, 512>>>((float4*)d, (long long)(n / 4)); });
#define RUNS(R, G, NT)                                                                  \
  time("run " #R " group " #G " nt " #NT, [&] {                                        \
    const int nblk = (T + R - 1) / R;                                                   \
    const int grid = G ? ((B + 7) / 8) * 8 * nblk : B * nblk;                           \
    runs<R, NT><<<grid, 512>>>(d, G);                                                   \
  });
  RUNS(8, 0, false) RUNS(8, 1, false) RUNS(8, 1, true)
  RUNS(16, 0, false) RUNS(16, 1, false)
  RUNS(32, 0, false) RUNS(32, 1, false) RUNS(32, 1, true)
  RUNS(64, 0, false) RUNS(64, 1, false)
#define WAVE4(W)                                                                        \
  time("wave4 x" #W " waves", [&] {                                                     \
    const int nblk = (T + 4 * W - 1) / (4 * W);                                         \
    wave4<W><<<((B + 7) / 8) * 8 * nblk, 64 * W>>>(d);                                  \
  });
  WAVE4(4) WAVE4(8) WAVE4(16)
  return 0;
}
