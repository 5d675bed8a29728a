"""Standard MIDI File reader and piano roll, for the score side of the path.

The reference reads scores with pretty_midi (`preprocess.py:146-147` load_midi,
`inference.py:40-41` process_custom_midi_and_audio):

    pianoroll = pretty_midi.PrettyMIDI(path).get_piano_roll(fs=wps).T

pretty_midi (and mido under it) is absent from this image and version-unpinned
by the reference, so this module restates the published behaviour of
pretty_midi 0.2.9/0.2.10 on top of a small SMF parser (parity unpinned; the
integer framing after it is bit-exact with the reference, see preprocess.py):

- ticks -> seconds: tempo changes are read from track 0 only, default 120 bpm,
  piecewise-linear tick scales accumulated segment by segment;
- instruments are keyed by (program, channel, track); channel 9 is drums;
- a note-off (or note-on with velocity 0) closes every open note of the same
  (channel, pitch) that did not start on the same tick; notes never closed are
  dropped; control changes go to their instrument (kept only if it has notes);
- Instrument.get_piano_roll: roll[pitch, int(start*fs):int(end*fs)] += velocity
  over int(fs*end_time) columns (end_time = last note end / control change),
  drums contribute zeros, then the sustain pedal (CC 64 >= pedal_threshold)
  holds the running maximum of each pitch between pedal-down and pedal-up;
- PrettyMIDI.get_piano_roll sums the instruments' rolls, padded to the longest.

The host parses files (I/O, a few KB); binarisation and onoff run on the device
(`preprocess.pianoroll_onoff`).
"""
import collections
import struct

import numpy as np

__all__ = ["Note", "ControlChange", "Instrument", "MidiFile", "read_midi", "get_piano_roll"]

Note = collections.namedtuple("Note", "velocity pitch start end")
ControlChange = collections.namedtuple("ControlChange", "number value time")

_DATA_LEN = {0x80: 2, 0x90: 2, 0xA0: 2, 0xB0: 2, 0xC0: 1, 0xD0: 1, 0xE0: 2}


class Instrument:
    def __init__(self, program, is_drum=False):
        self.program = program
        self.is_drum = is_drum
        self.notes = []
        self.control_changes = []

    def get_end_time(self):
        ev = [n.end for n in self.notes] + [c.time for c in self.control_changes]
        return max(ev) if ev else 0.0

    def get_piano_roll(self, fs=100, pedal_threshold=64):
        if not self.notes:
            return np.zeros((128, 0))
        roll = np.zeros((128, int(fs * self.get_end_time())))
        if self.is_drum:
            return roll
        for n in self.notes:
            roll[n.pitch, int(n.start * fs):int(n.end * fs)] += n.velocity
        if pedal_threshold is not None:
            t_on, down = 0, False
            for cc in self.control_changes:
                if cc.number != 64:
                    continue
                t_now = int(cc.time * fs)
                on = cc.value >= pedal_threshold
                if not down and on:
                    t_on, down = t_now, True
                elif down and not on:
                    sub = roll[:, t_on:t_now]
                    roll[:, t_on:t_now] = np.maximum.accumulate(sub, axis=1) if sub.size else sub
                    down = False
        return roll


def _vlq(buf, i):
    v = 0
    while True:
        if i >= len(buf):
            raise ValueError("truncated variable-length quantity")
        c = buf[i]
        i += 1
        v = (v << 7) | (c & 0x7F)
        if not c & 0x80:
            return v, i


def _parse_track(buf):
    """-> list of (abs_tick, kind, fields) with kind in note_on/note_off/cc/program/tempo."""
    ev, i, tick, status = [], 0, 0, None
    while i < len(buf):
        dt, i = _vlq(buf, i)
        tick += dt
        b = buf[i]
        if b == 0xFF:  # meta
            mtype = buf[i + 1]
            ln, i = _vlq(buf, i + 2)
            data = buf[i:i + ln]
            i += ln
            if mtype == 0x51 and ln == 3:
                ev.append((tick, "tempo", (data[0] << 16) | (data[1] << 8) | data[2]))
            elif mtype == 0x2F:
                break
            continue
        if b in (0xF0, 0xF7):  # sysex
            ln, i = _vlq(buf, i + 1)
            i += ln
            continue
        if b & 0x80:
            status = b
            i += 1
        elif status is None:
            raise ValueError("running status without a status byte")
        hi, ch = status & 0xF0, status & 0x0F
        if hi not in _DATA_LEN:
            raise ValueError("unsupported MIDI status 0x%02x" % status)
        d = buf[i:i + _DATA_LEN[hi]]
        i += _DATA_LEN[hi]
        if hi == 0x90 and d[1] > 0:
            ev.append((tick, "note_on", (ch, d[0], d[1])))
        elif hi in (0x80, 0x90):
            ev.append((tick, "note_off", (ch, d[0])))
        elif hi == 0xB0:
            ev.append((tick, "cc", (ch, d[0], d[1])))
        elif hi == 0xC0:
            ev.append((tick, "program", (ch, d[0])))
    return ev


class MidiFile:
    """pretty_midi.PrettyMIDI(path) restricted to what get_piano_roll reads."""

    def __init__(self, source):
        if isinstance(source, (bytes, bytearray)):
            data = bytes(source)
        else:
            with open(source, "rb") as f:
                data = f.read()
        if data[:4] != b"MThd":
            raise ValueError("not a Standard MIDI File")
        hlen, fmt, ntrk, div = struct.unpack(">IHHH", data[4:14])
        if div & 0x8000:
            raise ValueError("SMPTE time division is not supported")
        self.resolution = div
        i = 8 + hlen
        tracks = []
        while i + 8 <= len(data) and len(tracks) < ntrk:
            cid, ln = data[i:i + 4], struct.unpack(">I", data[i + 4:i + 8])[0]
            if cid == b"MTrk":
                try:
                    tracks.append(_parse_track(data[i + 8:i + 8 + ln]))
                except IndexError:
                    raise ValueError("truncated MTrk chunk") from None
            i += 8 + ln
        if not tracks:
            raise ValueError("no MTrk chunks")
        max_tick = max((e[0] for t in tracks for e in t), default=0) + 1
        self._tick_to_time = self._tick_map(tracks[0], max_tick)
        self.instruments = self._instruments(tracks)

    def _tick_map(self, track0, max_tick):
        scales = [(0, 60.0 / (120.0 * self.resolution))]
        for tick, kind, tempo in track0:
            if kind != "tempo":
                continue
            s = 60.0 / ((6e7 / tempo) * self.resolution)
            if tick == 0:
                scales = [(0, s)]
            elif s != scales[-1][1]:
                scales.append((tick, s))
        t2t = np.zeros(max_tick + 1)
        last_end = 0.0
        for n, (start, s) in enumerate(scales):
            end = scales[n + 1][0] if n + 1 < len(scales) else max_tick
            t2t[start:end + 1] = last_end + s * np.arange(end - start + 1)
            last_end = t2t[end]
        return t2t

    def _instruments(self, tracks):
        t2t = self._tick_to_time
        inst, stragglers = collections.OrderedDict(), {}

        def get(program, ch, track, create):
            key = (program, ch, track)
            if key in inst:
                return inst[key]
            if not create:
                return stragglers.setdefault(key, Instrument(program, ch == 9))
            ins = stragglers.pop(key, None) or Instrument(program, ch == 9)
            inst[key] = ins
            return ins

        for ti, track in enumerate(tracks):
            program = [0] * 16
            open_notes = collections.defaultdict(list)
            for tick, kind, f in track:
                if kind == "program":
                    program[f[0]] = f[1]
                elif kind == "note_on":
                    open_notes[(f[0], f[1])].append((tick, f[2]))
                elif kind == "note_off":
                    key = (f[0], f[1])
                    if key not in open_notes:
                        continue
                    close = [(s, v) for s, v in open_notes[key] if s != tick]
                    keep = [(s, v) for s, v in open_notes[key] if s == tick]
                    for s, v in close:
                        get(program[f[0]], f[0], ti, True).notes.append(
                            Note(v, f[1], float(t2t[s]), float(t2t[tick])))
                    if close and keep:
                        open_notes[key] = keep
                    else:
                        del open_notes[key]
                elif kind == "cc":
                    get(program[f[0]], f[0], ti, False).control_changes.append(
                        ControlChange(f[1], f[2], float(t2t[tick])))
        return list(inst.values())

    def get_piano_roll(self, fs=100, pedal_threshold=64):
        """(128, n) float64, summed over instruments (pretty_midi PrettyMIDI.get_piano_roll)."""
        if not self.instruments:
            return np.zeros((128, 0))
        rolls = [i.get_piano_roll(fs=fs, pedal_threshold=pedal_threshold) for i in self.instruments]
        out = np.zeros((128, max(r.shape[1] for r in rolls)))
        for r in rolls:
            out[:, :r.shape[1]] += r
        return out


def read_midi(source):
    return MidiFile(source)


def get_piano_roll(source, fs, pedal_threshold=64):
    """`pretty_midi.PrettyMIDI(source).get_piano_roll(fs=fs)` (preprocess.py:147)."""
    return MidiFile(source).get_piano_roll(fs=fs, pedal_threshold=pedal_threshold)
