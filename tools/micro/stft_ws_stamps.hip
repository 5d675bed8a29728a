// Dev tool: per-phase cycle stamps of the warp-specialised STFT kernel (stft_ws_kernel, config 2:
// 256 x 64,256 samples, hop 256, log-power). Mean cycles between consecutive stamps, separately
// for compute waves (0-7) and memory waves (8-11):
//   compute: 0 top, 1 after barrier A (span read), 2 windowed, 3 FFT done, 4 post-twist+staged,
//            5 after barrier B
//   memory:  0 top, 1 after barrier A, 2 DMA issued, 3 staging read, 4 stores + DMA wait,
//            5 after barrier B
#define STFT_STAMPS 1
#include "../../ml_music_style_transfer_amd/csrc/fft.hip"
#include <cstdio>
#include <vector>
int main() {
  const int B = 256, L = 64256, hop = 256, T = 1 + L / hop;
  float *x, *out;
  (void)hipMalloc(&x, (size_t)B * L * 4);
  (void)hipMalloc(&out, (size_t)B * NB * T * 4);
  std::vector<float> hx((size_t)B * L);
  for (size_t i = 0; i < hx.size(); ++i) hx[i] = 0.3f * sinf(0.01f * (float)(i % 9973)) + 1e-3f * (float)(i % 7);
  (void)hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 3; ++rep)
    if (mst_stft_logpow_f32(x, B, L, 2048, hop, 0, out, nullptr)) { printf("launch failed\n"); return 1; }
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, nullptr);
  for (int rep = 0; rep < 10; ++rep) mst_stft_logpow_f32(x, B, L, 2048, hop, 0, out, nullptr);
  (void)hipEventRecord(e1, nullptr);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> st(512 * 16 * 16 * 16);
  (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_stamps), st.size() * 8);
  printf("kernel %.4f ms (stamped build)\n", ms / 10);
  for (int role = 0; role < 2; ++role) {
    const int w0 = role ? 8 : 0, w1 = role ? 12 : 8;
    double acc[6] = {0}, loop = 0;
    long n = 0, nl = 0;
    for (int g = 0; g < 256; ++g)
      for (int w = w0; w < w1; ++w)
        for (int it = 1; it < 15; ++it) {
          const unsigned long long* s = &st[((g * 16 + w) * 16 + it) * 16];
          bool ok = true;
          for (int i = 0; i < 6; ++i) ok = ok && s[i];
          for (int i = 1; i < 6; ++i) ok = ok && s[i] >= s[i - 1];
          if (!ok) continue;
          for (int i = 1; i < 6; ++i) acc[i] += (double)(s[i] - s[i - 1]);
          ++n;
          const unsigned long long* nx = s + 16;
          if (nx[0] && nx[0] >= s[5]) { loop += (double)(nx[0] - s[0]); ++nl; }
        }
    printf("%s waves: %ld samples, mean iteration %.0f cycles\n", role ? "memory" : "compute", n, nl ? loop / nl : 0.0);
    const char* cn[6] = {"", "0->1 span read + barrier A", "1->2 window", "2->3 fft1024", "3->4 post-twist + stage", "4->5 barrier B"};
    const char* mn[6] = {"", "0->1 barrier A", "1->2 DMA issue", "2->3 staging reads", "3->4 stores + DMA wait", "4->5 barrier B"};
    for (int i = 1; i < 6; ++i) printf("  %-30s %8.0f\n", role ? mn[i] : cn[i], n ? acc[i] / n : 0.0);
  }
  return 0;
}
