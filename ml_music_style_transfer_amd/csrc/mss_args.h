// Arguments of the multi-scale spectral loss kernels (mss.hip), shared with the n = 2048 kernel in
// fft.hip, which reuses fft.hip's register-resident 1024-point FFT.
#pragma once
#include <hip/hip_runtime.h>

constexpr int MSS_RWIN = 4096;  // padded samples owned per workgroup

struct MssArgs {
  const float* pred;
  const float* target;
  long long L;
  int T, nwg;
  float alpha, eps, inv_cnt;
  const float* tmag;   // (B, T, n/2 + 1) target magnitudes |STFT_n(target)|, computed in float64
                       // by mss_target_kernel (mss.hip) and rounded to float
  float* dpred;        // (B, L) this size's gradient slab, or null
  float* edges;        // (B, n): gradient of the reflect-pad samples, head n/2 then tail n/2
  float* partial;      // (B, nwg, 2): per-workgroup sums of |dS| and |dlogS|
  float* spill;        // (B, nwg, 3n/4): the gradient a workgroup's last three frames put on the
                       // 3n/4 padded samples past its range (mss_sum_kernel and the edge fold add them)
};

// n = 2048: grid (nwg, B), 256 threads, one radix-2 step around two fft1024 (fft.hip)
void mss_fft2048_launch(const MssArgs& a, unsigned nwg, unsigned B, hipStream_t st);
