"""Host-side callers either side of the path: MIDI -> piano roll
(pretty_midi semantics, midi.py), WAV read/write (librosa.load / soundfile.write, wavio.py)
and the inference CLI's checkpoint resolution (inference.py:113-124).

pretty_midi, librosa and soundfile are absent here, so the expected values below are
computed by hand from their published rules: parity unpinned. The SMF bytes are built by
the small writer in this file, independently of the parser."""
import json
import os
import struct
import sys

import numpy as np
import pytest

from ml_music_style_transfer_amd import midi, wavio
from oracle import midi_ref


def _vlq(v):
    out = [v & 0x7F]
    v >>= 7
    while v:
        out.append(0x80 | (v & 0x7F))
        v >>= 7
    return bytes(reversed(out))


def _track(events):
    """events: (abs_tick, raw bytes); delta-encoded, end-of-track appended."""
    body, last = b"", 0
    for tick, raw in sorted(events, key=lambda e: e[0]):
        body += _vlq(tick - last) + raw
        last = tick
    body += _vlq(0) + b"\xff\x2f\x00"
    return b"MTrk" + struct.pack(">I", len(body)) + body


def _smf(tracks, division=480, fmt=1):
    return b"MThd" + struct.pack(">IHHH", 6, fmt, len(tracks), division) + b"".join(tracks)


def _tempo(bpm):
    us = int(round(6e7 / bpm))
    return b"\xff\x51\x03" + bytes([(us >> 16) & 255, (us >> 8) & 255, us & 255])


def _on(ch, p, v):
    return bytes([0x90 | ch, p, v])


def _off(ch, p):
    return bytes([0x80 | ch, p, 0])


def test_tempo_map_and_roll():
    """Tempo from track 0 (120 bpm, then 60 bpm at tick 960); notes on track 1."""
    t0 = _track([(0, _tempo(120)), (960, _tempo(60))])
    t1 = _track([(0, b"\xc0\x00"), (0, _on(0, 60, 100)), (480, _off(0, 60)),
                 (720, _on(0, 64, 80)), (1440, _off(0, 64))])
    m = midi.MidiFile(_smf([t0, t1]))
    notes = sorted(((n.pitch, n.start, n.end, n.velocity) for i in m.instruments for n in i.notes))
    # 120 bpm: 480 ticks = 0.5 s; after tick 960 (1.0 s) 60 bpm: 480 ticks = 1.0 s
    assert notes == [(60, 0.0, 0.5, 100), (64, 0.75, 2.0, 80)]
    roll = m.get_piano_roll(fs=172)
    np.testing.assert_array_equal(roll, midi_ref.piano_roll(notes, 172))
    assert roll.shape == (128, int(172 * 2.0))


def test_note_off_rules_and_running_status():
    """A note-off closes every open note of its (channel, pitch) not started on the same tick;
    note-on velocity 0 is a note-off; running status; unclosed notes are dropped."""
    raw = (_vlq(0) + bytes([0x90, 60, 90]) + _vlq(100) + bytes([60, 70])  # running status
           + _vlq(100) + bytes([60, 0])                                      # vel-0 off at 200
           + _vlq(0) + bytes([62, 50])                                       # on 62 at 200
           + _vlq(0) + b"\xff\x2f\x00")
    tr = b"MTrk" + struct.pack(">I", len(raw)) + raw
    m = midi.MidiFile(_smf([tr], division=100, fmt=0))
    notes = sorted((n.pitch, n.start, n.end, n.velocity) for i in m.instruments for n in i.notes)
    # 100 ticks per beat at 120 bpm: 1 tick = 5 ms. Both 60s close at tick 200; 62 never closes.
    assert notes == [(60, 0.0, 1.0, 90), (60, 0.5, 1.0, 70)]
    same_tick = _track([(0, _on(0, 60, 90)), (100, _on(0, 60, 70)), (100, _off(0, 60)),
                        (300, _off(0, 60))])
    m = midi.MidiFile(_smf([same_tick], division=100))
    notes = sorted((n.start, n.end, n.velocity) for i in m.instruments for n in i.notes)
    assert notes == [(0.0, 0.5, 90), (0.5, 1.5, 70)]


def test_sustain_pedal_and_drums():
    fs = 100
    tr = _track([(0, _on(0, 60, 100)), (48, _off(0, 60)),          # 0 .. 0.05 s
                 (24, bytes([0xB0, 64, 127])), (480, bytes([0xB0, 64, 0])),  # pedal .025-.5 s
                 (0, _on(9, 36, 120)), (960, _off(9, 36))])          # drum to 1.0 s
    m = midi.MidiFile(_smf([tr]))
    assert sorted(i.is_drum for i in m.instruments) == [False, True]
    roll = m.get_piano_roll(fs=fs)
    assert roll.shape == (128, 100)          # the drum extends the length, adds nothing
    assert roll[36].sum() == 0
    expect = np.zeros(100)
    expect[0:50] = 100                        # held by the pedal from frame 2 to frame 50
    np.testing.assert_array_equal(roll[60], expect)
    np.testing.assert_array_equal(m.get_piano_roll(fs=fs, pedal_threshold=None)[60][:10],
                                  np.r_[np.full(5, 100.0), np.zeros(5)])


def test_midi_errors():
    with pytest.raises(ValueError):
        midi.MidiFile(b"RIFF....")
    with pytest.raises(ValueError):
        midi.MidiFile(b"MThd" + struct.pack(">IHHH", 6, 0, 1, 0xE728))  # SMPTE


def test_wav_roundtrip_and_formats(tmp_path):
    rng = np.random.default_rng(0)
    y = (0.9 * np.sin(np.arange(4410) * 0.05) + 0.01 * rng.standard_normal(4410)).astype(np.float32)
    p = str(tmp_path / "a.wav")
    wavio.write(p, y, 44100)
    r, sr = wavio.load(p, sr=44100)
    assert sr == 44100 and r.dtype == np.float32 and r.shape == y.shape
    # libsndfile scales: write x * 0x7FFF, read int / 0x8000
    np.testing.assert_array_equal(r, (np.rint(y.astype(np.float64) * 32767) / 32768).astype(np.float32))
    wavio.write(p, np.array([2.0, -2.0], np.float32), 44100)
    np.testing.assert_array_equal(wavio.load(p)[0], np.array([32767, -32768]) / 32768.0)
    # stereo 24-bit PCM -> mono mean
    raw = np.array([[1 << 22, -(1 << 22)], [1 << 21, 1 << 21]], np.int32)
    b = b"".join(int(v & 0xFFFFFF).to_bytes(3, "little") for v in raw.ravel())
    fmt = struct.pack("<HHIIHH", 1, 2, 44100, 44100 * 6, 6, 24)
    wav = b"RIFF" + struct.pack("<I", 4 + 8 + 16 + 8 + len(b)) + b"WAVE" + b"fmt " + \
        struct.pack("<I", 16) + fmt + b"data" + struct.pack("<I", len(b)) + b
    q = tmp_path / "b.wav"
    q.write_bytes(wav)
    np.testing.assert_allclose(wavio.load(str(q))[0], [0.0, 0.25])
    with pytest.raises(ValueError):
        wavio.load(str(q), sr=16000)


def test_best_checkpoint_name(tmp_path):
    from ml_music_style_transfer_amd import inference
    with open(tmp_path / "hyperparams.json", "w") as f:
        json.dump({"best_epoch": 7, "best_loss": 0.5}, f)
    assert inference.best_checkpoint_name(str(tmp_path)) == "checkpoint-7.tar"


# ---------------------------------------------------------------- HDF5 data path (§8(f) #1)
def _split(rng, N=7, T=20, styles=("cuba", "upright")):
    pr = (rng.random((N, T, 128)) < 0.1).astype(float)
    oo = np.diff(np.concatenate([np.zeros((N, 1, 128)), pr], 1), axis=1)
    return pr, oo, {s: rng.random((N, 1025, T)) for s in styles}


def test_hdf5_schema_roundtrip_and_append(tmp_path):
    """io_manager.h5pyManager's layout: float64, chunked, resizable on axis 0, appended."""
    from ml_music_style_transfer_amd import h5
    rng = np.random.default_rng(1)
    a, b = rng.random((3, 20, 128)), rng.random((2, 20, 128))
    p = str(tmp_path / "x.hdf5")
    with h5.File(p, "w") as f:
        f.create_dataset("pianoroll", data=a, dtype="float64", maxshape=(None, 20, 128), chunks=True)
        d = f["pianoroll"]
        d.resize(d.shape[0] + b.shape[0], axis=0)
        d[-b.shape[0]:] = b
    with h5.File(p) as f:
        assert f.keys() == ["pianoroll"] and "pianoroll" in f and "onoff" not in f
        assert f["pianoroll"].shape == (5, 20, 128)
        np.testing.assert_array_equal(f["pianoroll"][:], np.concatenate([a, b]))
        np.testing.assert_array_equal(f["pianoroll"][:100], np.concatenate([a, b]))  # n_read > n
        np.testing.assert_array_equal(f["pianoroll"][3], b[0])
        with pytest.raises(KeyError):
            f["spec_cuba"]


def test_dataset_item_rule(tmp_path):
    """Dataseth5py.__getitem__ (train.py:74-99): concat+transpose, random style, random cond."""
    import random
    from ml_music_style_transfer_amd import data
    rng = np.random.default_rng(2)
    pr, oo, specs = _split(rng)
    data.write_split(str(tmp_path / "d_train.hdf5"), pr, oo, specs)
    ds = data.Dataseth5py(str(tmp_path / "d_train.hdf5"), n_read=5)
    assert ds.styles == ["spec_cuba", "spec_upright"] and len(ds) == 5
    random.seed(42)
    expect = []
    for i in (0, 4, 2):
        style = random.choice(ds.styles)
        r = random.randint(0, 4)
        expect.append((midi_ref.assemble_item(pr[i], oo[i]), specs[style[5:]][r], specs[style[5:]][i]))
    random.seed(42)
    for i, (eX, eC, eY) in zip((0, 4, 2), expect):
        X, Xc, y = ds[i]
        np.testing.assert_array_equal(X.numpy(), eX.astype(np.float32))
        np.testing.assert_array_equal(Xc.numpy(), eC.astype(np.float32))
        np.testing.assert_array_equal(y.numpy(), eY.astype(np.float32))


def test_device_loader_reproduces_dataloader(tmp_path):
    """DeviceLoader == DataLoader(Dataseth5py, shuffle=True) batch for batch over two epochs
    (same torch and random seeds); checked on CPU tensors here, on the GPU in
    test_gpu_inference.py."""
    import torch
    from ml_music_style_transfer_amd import data
    pr, oo, specs = _split(np.random.default_rng(3))
    data.write_split(str(tmp_path / "d_train.hdf5"), pr, oo, specs)
    for shuffle in (True, False):
        torch.manual_seed(5)
        ds = data.Dataseth5py(str(tmp_path / "d_train.hdf5"))
        dl = torch.utils.data.DataLoader(ds, batch_size=3, shuffle=shuffle)
        ref = [[t.clone() for t in b] for _ in range(2) for b in dl]
        torch.manual_seed(5)
        dl2 = data.DeviceLoader(data.Dataseth5py(str(tmp_path / "d_train.hdf5")), batch_size=3,
                                shuffle=shuffle, device="cpu")
        got = [b for _ in range(2) for b in dl2]
        assert len(dl2) == len(dl) == 3 and len(got) == len(ref) == 6
        for r, g in zip(ref, got):
            for a, b in zip(r, g):
                assert torch.equal(a, b)


def test_device_loader_target_audio_once_per_item(tmp_path):
    """DeviceLoader(target_audio=f): every batch's target carries f(target) row for row as
    `target.mst_audio`, f runs once per (style, item) over all epochs (the multi-scale loss's
    Griffin-Lim target is a constant of the item, train.make_loss), and the batches themselves are
    unchanged (same draws as without it)."""
    import torch
    from ml_music_style_transfer_amd import data
    pr, oo, specs = _split(np.random.default_rng(11), N=7)
    path = str(tmp_path / "d_train.hdf5")
    data.write_split(path, pr, oo, specs)
    calls = []

    def f(target):  # a stand-in for the Griffin-Lim reconstruction: any per-row map
        calls.append(target.shape[0])
        return target.sum(1) * 0.5 + target[:, 3]

    import random
    torch.manual_seed(2)
    random.seed(2)
    dl0 = data.DeviceLoader(data.Dataseth5py(path), batch_size=4, shuffle=True, device="cpu")
    plain = [b for _ in range(3) for b in dl0]
    torch.manual_seed(2)
    random.seed(2)
    dl = data.DeviceLoader(data.Dataseth5py(path), batch_size=4, shuffle=True, device="cpu",
                           target_audio=f)
    got = [b for _ in range(3) for b in dl]
    assert len(got) == len(plain) == 6
    for (x, c, y), (x0, c0, y0) in zip(got, plain):
        assert torch.equal(x, x0) and torch.equal(c, c0) and torch.equal(y, y0)
        assert torch.equal(y.mst_audio, f(y))
    drawn = dl._audio_done.sum()
    assert sum(calls[:-len(got)]) == drawn  # (the checks above called f once per batch too)
    assert drawn <= len(dl.styles) * dl.n


def test_musicnet_solo_piano_filter(tmp_path):
    """extract_piano_pieces_from_musicnet_dataset.py:10-24: keep label files whose only
    instrument is 1 (piano)."""
    from ml_music_style_transfer_amd import musicnet
    d = tmp_path / "test_labels"
    d.mkdir()
    rows = {"1759": [1, 1, 1], "2106": [1, 41, 1], "1819": [7, 7], "2303": [1]}
    for k, inst in rows.items():
        lines = ["start_time,end_time,instrument,note,start_beat,end_beat,note_value"]
        lines += ["%d,%d,%d,60,0.0,1.0,Quarter" % (i * 10, i * 10 + 5, v) for i, v in enumerate(inst)]
        (d / f"{k}.csv").write_text("\n".join(lines) + "\n")
    got = musicnet.main(str(tmp_path), "test", str(tmp_path / "piano_pieces"))
    assert sorted(got) == ["1759.csv", "2303.csv"]
    assert (tmp_path / "piano_pieces_test.txt").read_text().split() == got


def test_device_loader_distributed_shards(tmp_path):
    """DeviceLoader(sampler=DistributedSampler(ds, W, r)) == DataLoader(ds, sampler=...) for
    every rank and two epochs, and the ranks' shards cover the split (§8(e): one shard of the
    global batch per GPU)."""
    import random
    import torch
    from torch.utils.data.distributed import DistributedSampler
    from ml_music_style_transfer_amd import data
    pr, oo, specs = _split(np.random.default_rng(7), N=10)
    path = str(tmp_path / "d_train.hdf5")
    data.write_split(path, pr, oo, specs)
    W = 4
    seen = []
    for r in range(W):
        torch.manual_seed(3)
        ds = data.Dataseth5py(path)
        s1 = DistributedSampler(ds, num_replicas=W, rank=r, shuffle=True, seed=9)
        dl = torch.utils.data.DataLoader(ds, batch_size=2, sampler=s1)
        ref = []
        for ep in range(2):
            s1.set_epoch(ep)
            ref += [[t.clone() for t in b] for b in dl]
        torch.manual_seed(3)
        ds2 = data.Dataseth5py(path)
        s2 = DistributedSampler(ds2, num_replicas=W, rank=r, shuffle=True, seed=9)
        dl2 = data.DeviceLoader(ds2, batch_size=2, device="cpu", sampler=s2)
        got = []
        for ep in range(2):
            dl2.set_epoch(ep)
            got += list(dl2)
        assert len(dl2) == len(dl) == 2 and len(got) == len(ref) == 4
        for a3, b3 in zip(ref, got):
            for a, b in zip(a3, b3):
                assert torch.equal(a, b)
        s2.set_epoch(0)
        seen += list(iter(s2))
    assert sorted(set(seen)) == list(range(10))


def test_malformed_inputs_raise_valueerror(tmp_path):
    hdr = b"MThd" + struct.pack(">IHHH", 6, 0, 1, 480)
    with pytest.raises(ValueError):
        midi.MidiFile(hdr + b"MTrk" + struct.pack(">I", 3) + b"\x00\x90\x3c")  # cut mid-event
    fmt = struct.pack("<HHIIHH", 1, 1, 44100, 44100 * 2, 2, 12)
    wav = b"RIFF" + struct.pack("<I", 36) + b"WAVE" + b"fmt " + struct.pack("<I", 16) + fmt + \
        b"data" + struct.pack("<I", 0)
    (tmp_path / "c.wav").write_bytes(wav)
    with pytest.raises(ValueError):
        wavio.load(str(tmp_path / "c.wav"))


def test_preprocess_zip_data_dir(tmp_path):
    """preprocess.py:204-210: a zip -data-dir is extracted and replaced by its root directory;
    a plain directory passes through."""
    import zipfile
    from ml_music_style_transfer_amd import preprocess as PP
    zpath = tmp_path / "style_transfer_train.zip"
    with zipfile.ZipFile(zpath, "w") as zf:
        zf.writestr("style_transfer_train/2308_prelude18_mixcraft.mid", b"MThd")
        zf.writestr("style_transfer_train/2308_prelude18_harpsichord.wav", b"RIFF")
    out = tmp_path / "x"
    out.mkdir()
    d = PP.resolve_data_dir(str(zpath), extract_to=str(out))
    assert d == str(out / "style_transfer_train")
    assert sorted(os.listdir(d)) == ["2308_prelude18_harpsichord.wav", "2308_prelude18_mixcraft.mid"]
    assert PP.resolve_data_dir(d) == d


def test_bench_aux_parity_verdict_modes():
    """bench_aux's sampled oracle checks stop a standalone run on a miss (strict) but only record
    it when bench.py drives them, so one miss cannot cost the whole measured line."""
    import argparse

    import bench_aux
    assert bench_aux._verdict(True, "", argparse.Namespace(strict=True)) == {"ok": True}
    with pytest.raises(AssertionError):
        bench_aux._verdict(False, "miss", argparse.Namespace(strict=True))
    assert bench_aux._verdict(False, "miss", argparse.Namespace(strict=False)) == {"ok": False, "miss": "miss"}


def test_torch_fp32_mss_gap_matches_definition():
    """The tolerance basis of bench_aux's config-5 check: torch's fp32 multi-scale loss vs the
    float64 oracle (tiny case, CPU)."""
    import numpy as np

    import bench_aux
    from oracle import spectral_ref as SR
    rng = np.random.default_rng(0)
    q = (0.3 * np.sin(np.arange(3000) / 7.0)).astype(np.float32)
    p = (q + 0.05 * rng.standard_normal(3000)).astype(np.float32)
    ref, _ = SR.multiscale_spectral_loss_grad(p.astype(np.float64), q.astype(np.float64), 1.0, 1e-7, (256, 64))
    gap = bench_aux._torch_fp32_mss_gap(p, q, (256, 64), ref)
    assert 0.0 <= gap < 1e-3
