"""Drop-in for the reference synthesis path (model/inference.py) on the device.

`AudioSynthesizer(checkpoint, exp_dir, midi_source, audio_source)` and `main()`
keep the reference's constructor, CLI and file layout (inference.py:22-128):
`experiments/<exp-name>/hyperparams.json` -> best_epoch ->
`checkpoint-<best_epoch>.tar` ({'epoch', 'state_dict', 'optimizer'}, written by
train.main, train.py:202-208), the score from `<exp_dir>/midi/<midi-source>`,
the style audio from `<audio-source>`, and `output-<i>.wav` files in the first
free `audio_output_<id>` directory.

- Checkpoints load with `torch.load(..., weights_only=True)` (tensors and plain
  containers only) and `load_state_dict` into the flat-buffer PerformanceNet.
- MIDI and WAV parsing restate pretty_midi / librosa.load / soundfile.write
  (midi.py, wavio.py; parity unpinned, the libraries are absent here).
- The spectrogram (STFT log-power), the onoff roll, the model forward and
  Griffin-Lim all run on the device. `griffinlim` keeps the reference signature
  (inference.py:105-110): log-power in, sqrt(expm1(clip(S,0,20))) magnitude,
  librosa.griffinlim with momentum 0.99, as one device program per iteration
  (fft.hip). The reference's init='random' is unseeded; `seed` fixes it.
"""
import argparse
import json
import os

import numpy as np
import torch

from . import spectral
from . import wavio
from .model import PerformanceNet
from .preprocess import hp as pp_hp
from .preprocess import midi_file_to_roll, process_spectrum_from_chunk, read_audio


def load_checkpoint(path):
    """torch.load of a train.main checkpoint, executing nothing from the file."""
    return torch.load(path, map_location="cpu", weights_only=True)


def best_checkpoint_name(exp_dir):
    """inference.py:119-121: checkpoint-<best_epoch>.tar from hyperparams.json."""
    with open(os.path.join(exp_dir, 'hyperparams.json'), 'r') as hpfile:
        hp = json.load(hpfile)
    return 'checkpoint-{}.tar'.format(hp['best_epoch'])


class AudioSynthesizer():
    """inference.py:22-110."""

    def __init__(self, checkpoint=None, exp_dir=None, midi_source=None, audio_source=None,
                 n_iter=300, seed=0):
        self.exp_dir = exp_dir
        self.checkpoint = (load_checkpoint(os.path.join(exp_dir, checkpoint))
                           if checkpoint is not None and exp_dir is not None else None)
        self.sample_rate = pp_hp.sr
        self.wps = pp_hp.wps
        self.midi_source = midi_source
        self.audio_source = audio_source
        self.n_iter = n_iter
        self.seed = seed

    def get_test_midi(self):
        """inference.py:32-36."""
        X = np.load(os.path.join(self.exp_dir, 'test_data/test_X.npy'))
        rand = np.random.randint(len(X), size=5)
        return torch.from_numpy(np.stack([X[i] for i in rand]).astype(np.float32)).cuda()

    def process_custom_midi_and_audio(self, midi_filename, audio_filename):
        """inference.py:38-72: (pianoroll (1,128,T), onoff (1,128,T), spec (1,1025,T)) on the
        device. The score (wps frames/s) and the audio (1 + L//256 frames) rarely have the same
        length; the reference leaves that as a TODO (inference.py:62-68, its forward then fails
        in the first DenseConcat), here both are cut to the shorter one."""
        pianoroll, onoff = midi_file_to_roll(os.path.join(self.exp_dir, 'midi', midi_filename))
        audio = read_audio(audio_filename)
        spec = process_spectrum_from_chunk(torch.from_numpy(audio).cuda())
        T = min(pianoroll.shape[0], spec.shape[1])
        pianoroll = torch.from_numpy(pianoroll[:T].T.astype(np.float32)).cuda().unsqueeze(0)
        onoff = torch.from_numpy(onoff[:T].T.astype(np.float32)).cuda().unsqueeze(0)
        return pianoroll.contiguous(), onoff.contiguous(), spec[:, :T].contiguous().unsqueeze(0)

    def model(self):
        model = PerformanceNet().cuda()
        model.load_state_dict(self.checkpoint['state_dict'])
        return model

    def inference(self):
        """inference.py:74-91."""
        score, onoff, spec = self.process_custom_midi_and_audio(self.midi_source, self.audio_source)
        model = self.model()
        print('Inferencing spectrogram......')
        with torch.no_grad():
            model.eval()
            test_results = model(score, spec, onoff)
        output_dir = self.create_output_dir()
        audio = spectral.griffinlim(test_results, n_iter=self.n_iter, momentum=0.99,
                                    init="random", seed=self.seed, from_logpow=True).cpu().numpy()
        paths = []
        for i in range(len(audio)):
            paths.append(os.path.join(output_dir, 'output-{}.wav'.format(i + 1)))
            wavio.write(paths[-1], audio[i], self.sample_rate)
        return paths

    def create_output_dir(self):
        """inference.py:93-103."""
        dir_id = 1
        while True:
            try:
                audio_out_dir = os.path.join(self.exp_dir, 'audio_output_{}'.format(dir_id))
                os.makedirs(audio_out_dir)
                return audio_out_dir
            except FileExistsError:
                dir_id += 1

    def griffinlim(self, spectrogram, audio_id, n_iter=300, window='hann', n_fft=2048,
                   hop_length=256, verbose=False, seed=0):
        """inference.py:105-110. spectrogram: (1025, T) log-power (NumPy or tensor)."""
        if window != 'hann' or n_fft != 2048:
            raise ValueError("the reference path uses a 2048-point Hann window")
        is_np = not isinstance(spectrogram, torch.Tensor)
        S = torch.from_numpy(np.ascontiguousarray(spectrogram, np.float32)) if is_np else spectrogram
        S = S.cuda() if not S.is_cuda else S
        y = spectral.griffinlim(S.float(), n_iter=n_iter, hop_length=hop_length, momentum=0.99,
                                init="random", seed=seed, from_logpow=True)
        return y.cpu().numpy() if is_np else y

    def synthesize(self, model, score, spec, onoff, n_iter=300, seed=0):
        """model forward (no_grad, eval) then Griffin-Lim of every item (inference.py:74-91)."""
        with torch.no_grad():
            model.eval()
            out = model(score, spec, onoff)
        return spectral.griffinlim(out, n_iter=n_iter, momentum=0.99, init="random", seed=seed,
                                   from_logpow=True)


def parse_args(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("-exp-name", type=str, required=True)
    parser.add_argument("-midi-source", type=str, required=True)
    parser.add_argument("-audio-source", type=str, required=True)
    parser.add_argument("--n-iter", type=int, default=300)
    parser.add_argument("--seed", type=int, default=0)
    return parser.parse_args(argv)


def main(argv=None):
    """inference.py:113-124."""
    args = parse_args(argv)
    exp_dir = os.path.join(os.path.abspath('./experiments'), args.exp_name)
    synth = AudioSynthesizer(best_checkpoint_name(exp_dir), exp_dir, args.midi_source,
                             args.audio_source, n_iter=args.n_iter, seed=args.seed)
    return synth.inference()


if __name__ == "__main__":
    main()


__all__ = ["AudioSynthesizer", "PerformanceNet", "main", "best_checkpoint_name", "load_checkpoint"]
