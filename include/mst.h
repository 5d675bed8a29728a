/*
 * mst.h — C ABI of libmst_hip.so, the MI355X (gfx950) kernels behind the
 * spectrogram style-transfer training path of silburt/ML_Music_Style_Transfer.
 *
 * Every entry point:
 *   - takes plain device pointers, sizes and a hipStream_t passed as void*;
 *   - is stream-ordered and asynchronous (no host sync, no allocation), so it is
 *     safe inside hipGraph capture; workspaces are sized by *_workspace_size();
 *   - returns 0 on success, MST_EINVAL for bad shapes/arguments, or
 *     -(hipError_t) when the launch fails. No C++ exception crosses the ABI.
 * Tensors are fp32, contiguous, PyTorch NCL layout (batch, channel, time)
 * unless stated otherwise.
 *
 * Reference interfaces replaced (file:line in the reference repository):
 *   mst_stft_logpow_f32      preprocessing/preprocess.py:47-49  process_spectrum_from_chunk
 *   mst_stft_mel_f32         tests/plot_spec.py:20              librosa.feature.melspectrogram
 *   mst_stft_complex_f32,
 *   mst_istft_f32,
 *   mst_griffinlim_f32       model/inference.py:105-110, tests/test_griffinlim.py:23  librosa.griffinlim
 *   mst_mss_loss_*           README.md:23, model/train.py:119-123 (engel_loss stub; build-defined)
 *   mst_conv_fwd_f32         model/model.py:14-31,98-99,242    nn.Conv1d / nn.ConvTranspose1d / nn.Linear
 *                            forward AND input-gradient (dgrad) — all are this implicit GEMM
 *   mst_conv_wgrad_f32       weight gradients of the same layers (loss.backward(), train.py:140)
 *   mst_instnorm_lrelu_fwd_f32 / _bwd_f32
 *                            model/model.py:40-53,65-69,81-89   InstanceNorm1d + LeakyReLU(0.01) [+ MaxPool1d(2)]
 *   mst_l1_fwd_f32 / _bwd_f32, mst_mse_fwd_f32
 *                            model/train.py:132-135,140,158     nn.L1Loss fwd/bwd, nn.MSELoss (test)
 *   mst_adam_f32 / _ex_f32 / _dev_f32
 *                            model/train.py:188,143             optim.Adam(lr=1e-3)
 *   mst_onoff_f32            preprocessing/preprocess.py:148-155 piano-roll binarise + onset/offset
 *   mst_render_logpow_f32 / _bwd_f32
 *                            model/inference.py:109 sqrt(expm1(clip(S,0,20))) with a held phase:
 *                            the multi-scale loss as a training loss (README.md:23, train.py:119-123)
 */
#ifndef MST_H
#define MST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MST_OK 0
#define MST_EINVAL (-1000)

#define MST_ACT_NONE 0
#define MST_ACT_RELU 1
#define MST_ACT_LRELU 2

#define MST_PAD_REFLECT 0
#define MST_PAD_CONSTANT 1

/* One source of a (virtually concatenated) NCL input: channels [c_begin, c_begin+C)
 * of the virtual tensor live at p[b*sb + (c - c_begin)*sc + (t + off)], valid
 * when 0 <= t + off < T. Models torch.cat + crop_and_concat (model.py:71-78,103)
 * without materialising the concatenation. */
typedef struct mst_src {
  const float* p;
  int64_t sb;   /* batch stride (elements) */
  int32_t sc;   /* channel stride */
  int32_t C;    /* channels */
  int32_t T;    /* valid time length */
  int32_t off;  /* source time = virtual time + off */
} mst_src;

/* One NCL destination of a conv-like GEMM, rows [m_begin, m_begin+C). */
typedef struct mst_dst {
  float* p;
  int64_t sb;
  int32_t sc;
  int32_t C;
  int32_t T;            /* valid time length: stores with t+off outside [0,T) are dropped */
  int32_t off;          /* dst time = output time + off */
  const float* gate;    /* optional: v = gate[same index] > 0 ? v*gate_scale : 0 (ReLU/dropout bwd) */
  float gate_scale;
  int32_t pad_;
} mst_dst;

/* Conv-like implicit GEMM (forward of Conv1d/ConvTranspose1d/Linear and their dgrad):
 *   Y[b][m][t*ostride + ophase] = act( alpha * sum_{c,tap} A(m,c,tap) * X(b, c, a*t + beta + g*tap) + bias[m] )
 * with A(m,c,tap) = A[m*sAm + c*sAc + tap*sAt], X the virtual concat of src[0..1]
 * (zero outside [0, Tv)), t in [0, Tn), GEMM dims M x (B*Tn) x (Ctot*taps).
 * Optional dropout (keep with prob 1-p, scale 1/(1-p)) keyed by (seed, dst index); with seed_dev
 * set the key's seed is seed + *seed_dev, read on the device (a captured hipGraph advances
 * *seed_dev itself, so replays draw fresh masks). */
typedef struct mst_conv_desc {
  int32_t B, M, Tn, Ctot, taps;
  int32_t a, beta, g;        /* input time = a*t + beta + g*tap */
  int32_t Tv;                /* virtual input length */
  const float* A;
  int64_t sAm, sAc, sAt;
  mst_src src[2];            /* src[1].C == 0 when unused */
  int32_t ostride, ophase;
  mst_dst dst[2];            /* rows [0,dst[0].C) -> dst[0], the rest -> dst[1] */
  float alpha;
  const float* bias;         /* nullable, length M */
  int32_t act;               /* MST_ACT_* */
  float drop_p;              /* 0 = no dropout */
  uint64_t seed;
  int32_t splitk;            /* K schedule: 0 = auto (split-K or stream-K by a cost model),
                                n > 0 = split-K over n slabs, -1 = stream-K over one residency
                                wave (512 workgroups), n < -1 = stream-K over -n workgroups */
  int32_t pad_;
  const uint64_t* seed_dev;  /* nullable */
} mst_conv_desc;

/* Weight gradient of a conv-like layer:
 *   out[m*ldo + c*ldc + tap*ldt] (+)= scale * sum_{b,t} P[b][m][t] * X(b, c, a*t + beta + g*tap)
 * P: (B, M, Tk) NCL (contiguous in t), X: virtual concat of src (zero outside [0,Tv)).
 * ldc = ldt = 0 selects the torch weight layout (ldc = taps, ldt = 1); ldc = 1 is the
 * tap-major layout. accumulate != 0 adds to existing values. */
typedef struct mst_wgrad_desc {
  int32_t B, M, Tk, Ctot, taps;
  int32_t a, beta, g;
  int32_t Tv;
  const float* P;
  int64_t sPb;
  int32_t sPc;
  int32_t pad0_;
  mst_src src[2];
  float* out;
  int64_t ldo;
  float scale;
  int32_t accumulate;
  int32_t splitk;            /* K schedule, as mst_conv_desc.splitk */
  int32_t pad1_;
  int64_t ldc, ldt;          /* output strides per input channel / per tap (0, 0: torch layout) */
} mst_wgrad_desc;

/* ---- conv/linear GEMMs (MFMA f32) ---- */
size_t mst_conv_fwd_workspace_size(const mst_conv_desc* d);
int mst_conv_fwd_f32(const mst_conv_desc* d, float* workspace, size_t ws_bytes, void* stream);
size_t mst_wgrad_workspace_size(const mst_wgrad_desc* d);
int mst_conv_wgrad_f32(const mst_wgrad_desc* d, float* workspace, size_t ws_bytes, void* stream);

/* ---- InstanceNorm1d(eps) + LeakyReLU(slope) [+ MaxPool1d(2,2)] over rows of length T ----
 * y: (rows, T) conv outputs. a: normalised+activated (rows, T). pooled: (rows, T/2) or NULL.
 * mean/rstd: per-row statistics saved for backward (length rows). */
int mst_instnorm_lrelu_fwd_f32(const float* y, int64_t rows, int32_t T, float eps, float slope,
                               float* a, float* pooled, float* mean, float* rstd, void* stream);
/* dy = d/dy of the forward, given upstream grads of a (d_a, nullable) and of pooled
 * (d_pool0, d_pool1: nullable, summed). Recomputes z and the pool argmax from y.
 * rowsum (nullable, length rows): the sum over t of each written dy row, i.e. the producing
 * layer's bias gradient per (b, c) (reduce over b with mst_bias_grad_rows_f32). */
int mst_instnorm_lrelu_bwd_f32(const float* y, const float* mean, const float* rstd, int64_t rows,
                               int32_t T, float slope, const float* d_a, const float* d_pool0,
                               const float* d_pool1, float* dy, float* rowsum, void* stream);

/* db[c] (+)= sum_{b,t} dy[b][c][t] for an NCL tensor (B, C, T). */
int mst_bias_grad_f32(const float* dy, int32_t B, int32_t C, int32_t T, float scale, float* db,
                      int32_t accumulate, void* stream);
/* db[c] (+)= scale * sum_b rowsum[b*C + c] (row sums from mst_instnorm_lrelu_bwd_f32). */
int mst_bias_grad_rows_f32(const float* rowsum, int32_t B, int32_t C, float scale, float* db,
                           int32_t accumulate, void* stream);

/* ---- L1 / MSE loss (train.py:132-135,158): loss[0] = sum|pred - target| / n (or squared),
 * accumulated as double partials in a workspace of mst_l1_workspace_size(n) bytes. ---- */
size_t mst_l1_workspace_size(int64_t n);
int mst_l1_fwd_f32(const float* pred, const float* target, int64_t n, float* loss, void* workspace,
                   void* stream);
int mst_mse_fwd_f32(const float* pred, const float* target, int64_t n, float* loss, void* workspace,
                    void* stream);

/* nn.L1Loss backward: dx = gscale[0] * sign(pred - target) / n (gscale nullable = 1). */
int mst_l1_bwd_f32(const float* pred, const float* target, int64_t n, const float* gscale, float* dx,
                   void* stream);
/* LeakyReLU backward from the activation's output sign: dx = dy * (y > 0 ? 1 : slope). */
int mst_lrelu_bwd_f32(const float* dy, const float* y, int64_t n, float slope, float* dx,
                      void* stream);
/* ReLU + inverted dropout backward from the kept output h (DenseConcat, model.py:105-106):
 * out = h > 0 ? d * s : 0 with s = 1/(1-p). */
int mst_relu_gate_bwd_f32(const float* d, const float* h, int64_t n, float s, float* out,
                          void* stream);

/* ---- Adam over a flat parameter buffer (torch.optim.Adam semantics, no weight decay) ----
 * At step t (1-based): lr_step = lr / (1 - b1^t); bc2_sqrt = sqrt(1 - b2^t) (NOT its inverse);
 * one_minus_b1 = 1 - b1 and one_minus_b2 = 1 - b2 computed in double by the caller and rounded,
 * as torch does (1 - 0.999f in float would differ from torch's 0.001f by 1.3e-5 relative):
 *   m = m + one_minus_b1 (g - m);  v = b2 v + one_minus_b2 g^2;
 *   p -= lr_step * m / (sqrt(v) / bc2_sqrt + eps).
 * p, g, m, v: n floats each, 16-byte aligned, the same element order (any layout, shared). */
int mst_adam_f32(float* p, const float* g, float* m, float* v, int64_t n, float lr_step, float b2,
                 float one_minus_b1, float one_minus_b2, float eps, float bc2_sqrt, void* stream);
/* The same update over at most max_blocks 256-thread workgroups (grid-stride): a background
 * launch beside other kernels (one workgroup per CU leaves the GEMMs their occupancy). */
int mst_adam_ex_f32(float* p, const float* g, float* m, float* v, int64_t n, float lr_step,
                    float b2, float one_minus_b1, float one_minus_b2, float eps, float bc2_sqrt,
                    int32_t max_blocks, void* stream);
/* The same update with the step-dependent pair read from device memory: hyper[0] = lr_step,
 * hyper[1] = bc2_sqrt (2 floats). A captured hipGraph (graphs.GraphedTrainStep) computes them
 * on the device from its own step counter, so one recorded launch serves every step. */
int mst_adam_dev_f32(float* p, const float* g, float* m, float* v, int64_t n, const float* hyper,
                     float b2, float one_minus_b1, float one_minus_b2, float eps, void* stream);

/* ---- elementwise helpers ---- */
int mst_scale_f32(float* x, int64_t n, float s, void* stream);
int mst_fill_f32(float* x, int64_t n, float v, void* stream);

/* ---- front end: STFT (Hann periodic, center, pad_mode), one clip per row of x (B, L) ----
 * n_fft == 2048 and hop in {64..1024} supported by the LDS FFT; T = 1 + L/hop, F = n_fft/2 + 1.
 * logpow: out (B, F, T) = log1p(|X|^2); power: |X|^2; complex: out (B, F, T, 2) interleaved. */
int mst_stft_logpow_f32(const float* x, int32_t B, int32_t L, int32_t n_fft, int32_t hop,
                        int32_t pad_mode, float* out, void* stream);
int mst_stft_power_f32(const float* x, int32_t B, int32_t L, int32_t n_fft, int32_t hop,
                       int32_t pad_mode, float* out, void* stream);
int mst_stft_complex_f32(const float* x, int32_t B, int32_t L, int32_t n_fft, int32_t hop,
                         int32_t pad_mode, float* out, void* stream);
/* mel: out (B, n_mels, T) = W_mel @ |X|^2 with W_mel given sparsely per band:
 * band m covers bins [start[m], start[m] + len[m]) with weights w[woff[m] + i]. */
int mst_stft_mel_f32(const float* x, int32_t B, int32_t L, int32_t n_fft, int32_t hop,
                     int32_t pad_mode, const int32_t* start, const int32_t* len,
                     const int32_t* woff, const float* w, int32_t n_mels, float* out, void* stream);
/* iSTFT (librosa.istft, center=True): X (B, F, T, 2) -> y (B, hop*(T-1)). */
int mst_istft_f32(const float* X, int32_t B, int32_t F, int32_t T, int32_t hop, float* y,
                  void* stream);
/* Griffin-Lim (librosa.griffinlim): S (B, F, T) magnitudes, n_iter iterations with momentum;
 * angles0 (B, F, T, 2) unit phases or NULL (= all ones); y (B, hop*(T-1)).
 * mag_from_logpow != 0 applies sqrt(expm1(clip(S,0,20))) first (inference.py:109). */
size_t mst_griffinlim_workspace_size(int32_t B, int32_t F, int32_t T, int32_t hop);
int mst_griffinlim_f32(const float* S, int32_t B, int32_t F, int32_t T, int32_t hop, int32_t n_iter,
                       float momentum, const float* angles0, int32_t mag_from_logpow, float* y,
                       void* workspace, size_t ws_bytes, void* stream);

/* ---- multi-scale spectral loss (DDSP; README.md:23, stub train.py:119-123; build-defined) ----
 * pred, target (B, L) waveforms; sizes[n_sizes] FFT sizes, powers of two in [64, 2048], hop n/4,
 * periodic Hann, center + reflect pad (L > n/2). loss (1 device float) =
 *   sum_n mean|S_n(pred) - S_n(target)| + alpha mean|log(S_n(pred)+eps) - log(S_n(target)+eps)|
 * dpred (B, L) (nullable) receives d loss / d pred. sizes is a HOST array (<= 8 entries). */
size_t mst_mss_workspace_size(int64_t B, int64_t L, int32_t n_sizes, const int32_t* sizes);
int mst_mss_loss_f32(const float* pred, const float* target, int64_t B, int64_t L, int32_t n_sizes,
                     const int32_t* sizes, float alpha, float eps, float* loss, float* dpred,
                     void* workspace, size_t ws_bytes, void* stream);

/* ---- log-power spectrogram -> complex spectrum with a held phase (the multi-scale loss as a
 * training loss; inference.py:109's magnitude inversion):
 *   X[b][t][f] = sqrt(expm1(clip(S[b][f][t], 0, 20))) * P[b][t][f] / |P[b][t][f]|  (1 if |P| = 0)
 * S (B, F, T) log-power; P, X (B, T, F, 2) frame-major complex (mst_stft_complex_f32's layout).
 * _bwd: dS[b][f][t] = Re(conj(U) dX[b][t][f]) * e^S / (2 M) inside (0, 20), else 0. ---- */
int mst_render_logpow_f32(const float* S, const float* P, int32_t B, int32_t F, int32_t T, float* X,
                          void* stream);
int mst_render_logpow_bwd_f32(const float* S, const float* P, const float* dX, int32_t B, int32_t F,
                              int32_t T, float* dS, void* stream);

/* ---- piano roll (preprocess.py:148-155): roll (B, T, 128) velocities ->
 *      binarised roll and onoff, both (B, T, 128) ---- */
int mst_onoff_f32(const float* roll, int32_t B, int32_t T, float* bin, float* onoff, void* stream);

/* library identity / sanity */
const char* mst_version(void);
/* MFMA products per fp32 multiply-add in the GEMMs: 6 = bf16x6 (fp32 operands split exactly
 * into three bf16 pieces, six bf16 MFMA products, fp32 accumulation). */
int mst_gemm_products(void);
int mst_device_arch(char* buf, int32_t n); /* writes gcnArchName of the current device */

#ifdef __cplusplus
}
#endif
#endif /* MST_H */
