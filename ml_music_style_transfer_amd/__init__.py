"""MI355X-native spectrogram style-transfer training path (silburt/ML_Music_Style_Transfer).

Drop-ins for the reference's hot path:
  model.PerformanceNet (+ blocks)        <- model/model.py
  train.train / train.test / Adam        <- model/train.py
  preprocess.process_spectrum_from_chunk <- preprocessing/preprocess.py
  inference.griffinlim                   <- model/inference.py
backed by hand-written gfx950 HIP kernels in libmst_hip.so (C ABI: include/mst.h).
"""
from . import _lib  # noqa: F401

__all__ = ["model", "train", "preprocess", "inference", "spectral", "engine", "kernels"]
