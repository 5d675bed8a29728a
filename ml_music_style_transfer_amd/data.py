"""Training data path: the reference's HDF5 dataset and a loader that keeps it in HBM.

`Dataseth5py` and `Process_Data` are drop-ins for train.py:45-116: same files
(`<data_dir>_train.hdf5` / `_test.hdf5`, schema in h5.py), same `n_read` prefix reads, same
item rule (X = concat(pianoroll, onoff, -1).T (256, T); style = random.choice(styles);
X_cond = spec_<style>[random.randint(0, n-1)]; y = spec_<style>[index]) drawn from Python's
global `random` seeded with 42, so the same items come out in the same order.

The reference builds every item with its own host->device copies (train.py:94-96), which its
TODO (train.py:53-57) names as the bottleneck after the HDF5 read. `DeviceLoader` is the
MI355X layout of the same data: the whole split is uploaded once as float32
(roll+onoff (N, 256, T), specs (S, N, 1025, T); the reference's ~1,700 chunks x 5 styles at
T=860 are ~30 GB, a tenth of one GPU's HBM) and each batch is three device gathers driven by
2 x B indices. It reproduces `DataLoader(Dataseth5py(...), batch_size, shuffle)` batch for
batch: the same RandomSampler permutation from torch's global generator and the same
per-item `random` draws, in the same order. With `sampler=DistributedSampler(dataset, W, r)`
each data-parallel rank keeps only its shard's batches (the split is still resident on every
GPU: one upload, no per-step host traffic), as DataLoader(..., sampler=...) would give.
"""
import random

import numpy as np
import torch

from . import h5

__all__ = ["Dataseth5py", "Process_Data", "DeviceLoader", "write_split", "h5pyManager"]


class Dataseth5py(torch.utils.data.Dataset):
    """train.py:45-104."""

    def __init__(self, in_file, seed=42, n_read=None, n_read_memory=None):
        super(Dataseth5py, self).__init__()
        self.dataset = h5.File(in_file, 'r')
        self.styles = [name for name in self.dataset.keys() if 'spec_' in name]
        rows = slice(None, n_read)
        self.pianoroll = self.dataset['pianoroll'][rows]
        self.onoff = self.dataset['onoff'][rows]
        self.specs = {}
        for style in self.styles:
            print(f"loading style: {style}")
            self.specs[style] = self.dataset[style][rows]
        self.n_data = self.pianoroll.shape[0]
        random.seed(seed)

    def __getitem__(self, index):
        pianoroll = np.concatenate((self.pianoroll[index], self.onoff[index]), axis=-1)
        pianoroll = np.transpose(pianoroll, (1, 0))
        style = random.choice(self.styles)
        spec = self.specs[style][index]
        rand_index = random.randint(0, self.n_data - 1)
        spec_rand = self.specs[style][rand_index]
        return torch.Tensor(pianoroll), torch.Tensor(spec_rand), torch.Tensor(spec)

    def __len__(self):
        return self.n_data


def Process_Data(data_dir, n_train_read=None, n_test_read=None, batch_size=16, device_resident=True):
    """train.py:107-116. With device_resident (default) the loaders are DeviceLoaders over the
    same datasets; False gives the reference's torch DataLoaders."""
    print("loading training data")
    train_dataset = Dataseth5py(data_dir + '_train.hdf5', n_read=n_train_read)
    print("loading test data")
    test_dataset = Dataseth5py(data_dir + '_test.hdf5', n_read=n_test_read)
    if device_resident:
        return (DeviceLoader(train_dataset, batch_size=batch_size, shuffle=True),
                DeviceLoader(test_dataset, batch_size=batch_size))
    return (torch.utils.data.DataLoader(train_dataset, batch_size=batch_size, shuffle=True),
            torch.utils.data.DataLoader(test_dataset, batch_size=batch_size))


class DeviceLoader:
    """DataLoader(dataset, batch_size, shuffle) over a Dataseth5py whose arrays live in HBM."""

    def __init__(self, dataset, batch_size=16, shuffle=False, device="cuda", sampler=None,
                 target_audio=None):
        self.dataset = dataset
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.sampler = sampler  # e.g. torch DistributedSampler: one rank's shard per process
        self.device = torch.device(device)
        # target_audio (optional): a map from a (b, 1025, T) batch of target spectrograms to its
        # (b, L) waveforms (the multi-scale loss's Griffin-Lim target, train.make_loss). Each
        # item's waveform is a constant of the item, so it is computed once, the first time the
        # item is drawn, and kept in HBM; every batch's target then carries its rows as
        # `target.mst_audio` (a device gather).
        self.target_audio = target_audio
        self._audio = None   # (styles, n, L) device buffer, allocated on first use
        self._audio_done = None
        ds = dataset
        self.n = ds.n_data
        self.styles = list(ds.styles)
        short = [s for s in self.styles if ds.specs[s].shape[0] != self.n]
        if short or not self.styles:
            # get_data skips a style whose audio is missing for a song, so its rows no longer
            # line up with pianoroll[i]; the reference then fails (or mismatches) per item
            raise ValueError(f"spec datasets {short or self.styles} do not have {self.n} rows")
        x = np.concatenate((ds.pianoroll, ds.onoff), axis=-1).astype(np.float32)
        self.X = torch.from_numpy(x).to(self.device).transpose(1, 2).contiguous()
        self.S = torch.empty((len(self.styles), self.n) + tuple(ds.specs[self.styles[0]].shape[1:]),
                             dtype=torch.float32, device=self.device)
        for i, s in enumerate(self.styles):
            self.S[i].copy_(torch.from_numpy(ds.specs[s].astype(np.float32)))

    def __len__(self):
        n = len(self.sampler) if self.sampler is not None else self.n
        return (n + self.batch_size - 1) // self.batch_size

    def set_epoch(self, epoch):
        if self.sampler is not None and hasattr(self.sampler, "set_epoch"):
            self.sampler.set_epoch(epoch)

    def _order(self):
        # torch.utils.data: every iterator draws its base seed from the global generator, then
        # a RandomSampler draws its own seed from it; the permutation comes from a generator
        # seeded with that. A given sampler (DistributedSampler) supplies the order itself.
        torch.empty((), dtype=torch.int64).random_()
        if self.sampler is not None:
            return list(iter(self.sampler))
        if not self.shuffle:
            return list(range(self.n))
        seed = int(torch.empty((), dtype=torch.int64).random_().item())
        g = torch.Generator()
        g.manual_seed(seed)
        return torch.randperm(self.n, generator=g).tolist()

    def __iter__(self):
        order = self._order()
        for b0 in range(0, len(order), self.batch_size):
            idx = order[b0:b0 + self.batch_size]
            sty, rnd = [], []
            for _ in idx:  # the per-item draws of Dataseth5py.__getitem__, in order
                sty.append(self.styles.index(random.choice(self.styles)))
                rnd.append(random.randint(0, self.n - 1))
            t = torch.tensor([idx, sty, rnd], dtype=torch.int64).to(self.device, non_blocking=True)
            target = self.S[t[1], t[0]]
            if self.target_audio is not None:
                target.mst_audio = self._target_audio(idx, sty, t, target)
            yield self.X[t[0]], self.S[t[1], t[2]], target

    def _target_audio(self, idx, sty, t, target):
        if self._audio_done is None:
            self._audio_done = np.zeros((len(self.styles), self.n), dtype=bool)
        miss = [j for j, (i, s) in enumerate(zip(idx, sty)) if not self._audio_done[s, i]]
        # an item drawn twice in one batch is computed once
        first = {}
        for j in miss:
            first.setdefault((sty[j], idx[j]), j)
        if first:
            rows = torch.tensor(sorted(first.values()), dtype=torch.int64, device=self.device)
            wav = self.target_audio(target[rows])
            if self._audio is None:
                self._audio = torch.empty((len(self.styles), self.n, wav.shape[-1]),
                                          dtype=wav.dtype, device=self.device)
            self._audio[t[1][rows], t[0][rows]] = wav
            for (s, i) in first:
                self._audio_done[s, i] = True
        return self._audio[t[1], t[0]]


def write_split(path, pianoroll, onoff, specs):
    """preprocess.get_data's output for one split (io_manager.h5pyManager): float64 datasets,
    chunked, resizable on axis 0. specs: {style: (N, 1025, T)}."""
    with h5.File(path, 'w') as f:
        for name, arr in [("pianoroll", pianoroll), ("onoff", onoff)] + \
                [("spec_" + s, a) for s, a in specs.items()]:
            a = np.asarray(arr, np.float64)
            f.create_dataset(name, data=a, dtype='float64', maxshape=(None,) + a.shape[1:],
                             chunks=True)


class h5pyManager():
    """preprocessing/utils/io_manager.py:39-76: create on first write, then resize on axis 0
    and append, so pianoroll[i] / onoff[i] / spec_<style>[i] line up."""

    def __init__(self, data):
        self.data = data

    def _append(self, name, arr):
        arr = np.asarray(arr, np.float64)
        if name not in self.data:
            self.data.create_dataset(name, data=arr, dtype='float64',
                                     maxshape=(None,) + arr.shape[1:], chunks=True)
        else:
            d = self.data[name]
            d.resize(d.shape[0] + arr.shape[0], axis=0)
            d[-arr.shape[0]:] = arr

    def write_pianoroll(self, pianoroll_list, onoff_list):
        self._append("pianoroll", pianoroll_list)
        self._append("onoff", onoff_list)

    def write_spectrum(self, spec_list, style):
        self._append(f'spec_{style}', spec_list)
