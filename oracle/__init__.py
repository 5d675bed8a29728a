"""Parity oracle — TEST INFRASTRUCTURE, NOT PRODUCT CODE.

CPU restatements of the reference's hot path (silburt/ML_Music_Style_Transfer):
  detinit.py       deterministic hash-based weights/inputs shared by fixtures and tests
  model_ref.py     PerformanceNet forward/L1/Adam (model/model.py, model/train.py) on torch-CPU
  spectral_ref.py  librosa stft/istft/griffinlim/mel semantics in float64 NumPy
                   (preprocessing/preprocess.py:47-57, model/inference.py:105-110,
                   tests/test_griffinlim.py:23, tests/plot_spec.py:20)
  midi_ref.py      framing constants, chunk formulas, piano-roll/onoff rules
                   (preprocessing/preprocess.py:17-42, 60-96, 118-160)

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
anything here, and only as the checker / CPU baseline. The product package
(ml_music_style_transfer_amd) never imports it and fails loudly without its HIP library.

Pinning: model_ref is pinned to the real reference by tests/golden/*.npz, made by
tests/golden/make_golden.py importing /root/reference/model/model.py in the build
container. librosa/pretty_midi are absent from every interpreter here, so
spectral_ref/midi_ref are restatements of the libraries' published algorithms
 cross-checked against torch.stft/istft (an independent
pocketfft path): "parity unpinned" against librosa itself.
"""
