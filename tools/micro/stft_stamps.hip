// Dev tool: per-phase cycle stamps of the frequency-major STFT kernel (config 2: 256 x 64,256
// samples, hop 256, log-power). Builds fft.hip with STFT_STAMPS and prints, per phase, the mean
// cycles (s_memtime) between consecutive stamps of wave 0..7 over all blocks.
//   stamps: 0 block start, 1 windowed, 2 frame done, 3 after 1st barrier, 4 staged (after 2nd
//           barrier), 5 written, 6 after last barrier
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
  std::vector<unsigned long long> st(512 * 16 * 16 * 16);
  (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_stamps), st.size() * 8);
  double acc[8] = {0}, tot = 0;
  long n[8] = {0};
  long nblocks = 0;
  const int NS = 7;
  for (int g = 0; g < 512; ++g)
    for (int w = 0; w < 16; ++w)
      for (int it = 0; it < 16; ++it) {
        const unsigned long long* s = &st[((g * 16 + w) * 16 + it) * 16];
        if (s[0] == 0 || s[NS - 1] == 0) continue;
        ++nblocks;
        for (int i = 1; i < NS; ++i)
          if (s[i] && s[i - 1] && s[i] >= s[i - 1]) { acc[i] += (double)(s[i] - s[i - 1]); ++n[i]; }
        const unsigned long long* nx = it + 1 < 16 ? s + 16 : nullptr;
        if (nx && nx[0]) { acc[0] += (double)(nx[0] - s[NS - 1]); ++n[0]; }
        tot += (double)(s[NS - 1] - s[0]);
      }
  const char* nm[7] = {"6->next 0 (loop)", "0->1 wait+window", "1->2 fft+post", "2->3 barrier",
                       "3->4 prefetch+stage+barrier", "4->5 write-out", "5->6 barrier"};
  printf("blocks stamped %ld, mean block %.0f cycles\n", nblocks, tot / (nblocks ? nblocks : 1));
  for (int i = 1; i < NS; ++i) printf("%-40s %8.0f\n", nm[i], n[i] ? acc[i] / n[i] : 0.0);
  printf("%-40s %8.0f\n", nm[0], n[0] ? acc[0] / n[0] : 0.0);
  // split of 3->4: 3->7 prefetch issue, 7->8 staging writes (lgkmcnt drained), 8->4 barrier
  double a1 = 0, a2 = 0, a3 = 0;
  long m = 0;
  for (int g = 0; g < 512; ++g)
    for (int w = 0; w < 16; ++w)
      for (int it = 0; it < 16; ++it) {
        const unsigned long long* s = &st[((g * 16 + w) * 16 + it) * 16];
        if (!s[3] || !s[7] || !s[8] || !s[4]) continue;
        a1 += (double)(s[7] - s[3]); a2 += (double)(s[8] - s[7]); a3 += (double)(s[4] - s[8]); ++m;
      }
  if (m) printf("  3->7 prefetch issue %.0f, 7->8 staging writes %.0f, 8->4 barrier %.0f\n", a1 / m, a2 / m, a3 / m);
  return 0;
}
