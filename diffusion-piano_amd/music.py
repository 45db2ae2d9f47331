"""Song ingestion for the batched piano environment (host precompute, init-time only).

Restates, without note_seq / pretty_midi (absent on the GPU box), the pieces of the
reference's music pipeline that feed the hot path:

* Standard MIDI File parsing with pretty_midi's note-pairing semantics
  (used by ``note_seq.midi_io.midi_file_to_note_sequence``, called at
  ``robopianist/music/midi_file.py:179`` and ``data_processing/add_fingering_to_midi.py:68``).
* ``MidiFile.trim_silence`` (``robopianist/music/midi_file.py:231-237``) with
  ``note_seq.sequences_lib.extract_subsequence`` semantics.
* ``NoteTrajectory.seq_to_trajectory`` (``robopianist/music/midi_file.py:315-362``) over the
  piano roll of ``robopianist/music/piano_roll.py:59-204`` (onset_window=0).
* ``add_fingering_from_annotation_file`` (``data_processing/add_fingering_to_midi.py:26-83``).
* ``twinkle_twinkle_little_star_one_hand`` (``robopianist/music/library.py:69-97``).

The product of this module is a :class:`SongTables` object: the dense per-control-step
goal table ``[T, 89]`` plus per-step (key, finger) lists that the GPU kernel reads.
"""

from __future__ import annotations

import math
import re
import struct
from dataclasses import dataclass, field
from pathlib import Path
from typing import List, Optional, Sequence, Tuple

import numpy as np

MIN_MIDI_PITCH_PIANO = 21  # robopianist/music/constants.py:21
MAX_MIDI_PITCH_PIANO = 108
NUM_KEYS = 88
MAX_VELOCITY = 127
SUSTAIN_PEDAL_CC_NUMBER = 64  # robopianist/music/constants.py:54
MAX_CC_VALUE = 127

# Maximum number of simultaneous notes per control step the device tables hold.
MAX_NOTES_PER_STEP = 16


@dataclass
class Note:
    pitch: int
    start_time: float
    end_time: float
    velocity: int = 80
    part: int = 0  # protobuf default: 0 (fingering is stored in `part`).


@dataclass
class ControlChange:
    time: float
    control_number: int
    control_value: int


@dataclass
class NoteSequence:
    notes: List[Note] = field(default_factory=list)
    control_changes: List[ControlChange] = field(default_factory=list)
    total_time: float = 0.0
    title: str = ""

    def has_fingering(self) -> bool:
        """``MidiFile.has_fingering`` (robopianist/music/midi_file.py:252-261)."""
        parts = {n.part for n in self.notes}
        return len(parts) > 1 and any(p != 0 for p in parts)


# ---------------------------------------------------------------------------------------
# Standard MIDI File parsing (pretty_midi semantics).
# ---------------------------------------------------------------------------------------


def _read_varlen(data: bytes, pos: int) -> Tuple[int, int]:
    value = 0
    while True:
        b = data[pos]
        pos += 1
        value = (value << 7) | (b & 0x7F)
        if not b & 0x80:
            return value, pos


def parse_midi(path) -> NoteSequence:
    """Parses a type-0/1 SMF into a :class:`NoteSequence`.

    Note pairing follows pretty_midi ``PrettyMIDI._load_instruments``: a note-off (or a
    note-on with velocity 0) closes every open note of that (channel, pitch) that started
    at an earlier tick; an open note started at the same tick stays open. Instruments are
    keyed by (track, channel, program) in first-seen order and their notes are appended
    instrument by instrument, which is the order note_seq copies them into the sequence.
    Ticks map to seconds through the merged tempo map (default 120 qpm).
    """
    data = Path(path).read_bytes()
    if data[:4] != b"MThd":
        raise ValueError(f"{path}: not a Standard MIDI File")
    hdr_len = struct.unpack(">I", data[4:8])[0]
    fmt, ntracks, division = struct.unpack(">HHH", data[8:14])
    if division & 0x8000:
        raise ValueError("SMPTE time division is not supported")
    pos = 8 + hdr_len

    tracks = []  # list of [(abs_tick, kind, payload)]
    for _ in range(ntracks):
        if data[pos:pos + 4] != b"MTrk":
            raise ValueError("bad track chunk")
        length = struct.unpack(">I", data[pos + 4:pos + 8])[0]
        p, end = pos + 8, pos + 8 + length
        tick, status, events = 0, 0, []
        while p < end:
            delta, p = _read_varlen(data, p)
            tick += delta
            b = data[p]
            if b == 0xFF:  # meta
                mtype = data[p + 1]
                mlen, p = _read_varlen(data, p + 2)
                payload = data[p:p + mlen]
                p += mlen
                if mtype == 0x51:
                    events.append((tick, "tempo", (payload[0] << 16) | (payload[1] << 8) | payload[2]))
                elif mtype == 0x2F:
                    break
                continue
            if b in (0xF0, 0xF7):  # sysex
                slen, p = _read_varlen(data, p + 1)
                p += slen
                continue
            if b & 0x80:
                status = b
                p += 1
            kind = status & 0xF0
            ch = status & 0x0F
            if kind in (0xC0, 0xD0):
                d1 = data[p]
                p += 1
                if kind == 0xC0:
                    events.append((tick, "program", (ch, d1)))
                continue
            d1, d2 = data[p], data[p + 1]
            p += 2
            if kind == 0x90:
                events.append((tick, "on" if d2 > 0 else "off", (ch, d1, d2)))
            elif kind == 0x80:
                events.append((tick, "off", (ch, d1, d2)))
            elif kind == 0xB0:
                events.append((tick, "cc", (ch, d1, d2)))
        tracks.append(events)
        pos = end

    # Tempo map (pretty_midi reads tempo changes from every track).
    tempos = sorted((t, v) for events in tracks for (t, k, v) in events if k == "tempo")
    if not tempos or tempos[0][0] != 0:
        tempos.insert(0, (0, 500000))
    # Collapse same-tick changes: the last one wins.
    tmap = []
    for t, v in tempos:
        if tmap and tmap[-1][0] == t:
            tmap[-1] = (t, v)
        else:
            tmap.append((t, v))
    seg_start_time = [0.0]
    for i in range(1, len(tmap)):
        dt_ticks = tmap[i][0] - tmap[i - 1][0]
        seg_start_time.append(seg_start_time[-1] + dt_ticks * tmap[i - 1][1] / 1e6 / division)

    def tick_to_time(tick: int) -> float:
        i = len(tmap) - 1
        while tmap[i][0] > tick:
            i -= 1
        return seg_start_time[i] + (tick - tmap[i][0]) * tmap[i][1] / 1e6 / division

    instruments = {}  # (track, channel, program) -> list of notes, insertion ordered
    ccs: List[ControlChange] = []
    for ti, events in enumerate(tracks):
        program = {}
        open_notes = {}
        for tick, kind, payload in events:
            if kind == "program":
                ch, prog = payload
                program[ch] = prog
            elif kind == "on":
                ch, pitch, vel = payload
                open_notes.setdefault((ch, pitch), []).append((tick, vel))
            elif kind == "off":
                ch, pitch, _ = payload
                key = (ch, pitch)
                if key not in open_notes:
                    continue
                to_close = [(s, v) for s, v in open_notes[key] if s != tick]
                to_keep = [(s, v) for s, v in open_notes[key] if s == tick]
                inst = instruments.setdefault((ti, ch, program.get(ch, 0)), [])
                for s, v in to_close:
                    inst.append(Note(pitch, tick_to_time(s), tick_to_time(tick), v))
                if to_close and to_keep:
                    open_notes[key] = to_keep
                elif to_close:
                    del open_notes[key]
            elif kind == "cc":
                ch, num, val = payload
                ccs.append(ControlChange(tick_to_time(tick), num, val))
    seq = NoteSequence(title=Path(path).stem)
    for notes in instruments.values():
        seq.notes.extend(notes)
    seq.control_changes = ccs
    seq.total_time = max([n.end_time for n in seq.notes] + [0.0])
    return seq


def trim_silence(seq: NoteSequence) -> NoteSequence:
    """``MidiFile.trim_silence``: ``extract_subsequence(seq, notes[0].start, notes[-1].end)``.

    note_seq semantics: notes are visited sorted by start time; notes starting inside
    ``[start, end)`` are shifted by ``-start`` and their end clipped to ``end``; the total
    time becomes the latest clipped end. Control changes inside the window are shifted;
    a sustain pedal held at ``start`` is re-emitted at time 0.
    """
    if not seq.notes:
        return NoteSequence(title=seq.title)
    start, end = seq.notes[0].start_time, seq.notes[-1].end_time
    out = NoteSequence(title=seq.title)
    for n in sorted(seq.notes, key=lambda n: n.start_time):
        if n.start_time < start or n.start_time >= end:
            continue
        e = min(n.end_time, end) - start
        out.notes.append(Note(n.pitch, n.start_time - start, e, n.velocity, n.part))
        out.total_time = max(out.total_time, e)
    pedal_value = None
    for cc in sorted(seq.control_changes, key=lambda c: c.time):
        if cc.time < start:
            if cc.control_number == SUSTAIN_PEDAL_CC_NUMBER:
                pedal_value = cc.control_value
            continue
        if cc.time >= end:
            continue
        out.control_changes.append(ControlChange(cc.time - start, cc.control_number, cc.control_value))
    if pedal_value is not None and pedal_value >= 64:
        out.control_changes.insert(0, ControlChange(0.0, SUSTAIN_PEDAL_CC_NUMBER, pedal_value))
    return out


_NOTE_VALUES = {
    "C": 0, "C#": 1, "Db": 1, "D": 2, "D#": 3, "Eb": 3, "E": 4, "F": 5, "F#": 6,
    "Gb": 6, "G": 7, "G#": 8, "Ab": 8, "A": 9, "A#": 10, "Bb": 10, "B": 11,
}


def parse_pitch_to_midi_number(pitch_str: str) -> int:
    """``data_processing/add_fingering_to_midi.py:7-24``."""
    m = re.match(r"([A-G][#b]?)(\d+)", pitch_str)
    if not m:
        raise ValueError(f"Invalid pitch format: {pitch_str}")
    note, octave = m.groups()
    return _NOTE_VALUES[note] + (int(octave) + 1) * 12


def add_fingering_from_annotation_file(midi_path, annotation_path) -> NoteSequence:
    """``data_processing/add_fingering_to_midi.py:26-83``.

    Each sequence note takes the finger of the first annotation line whose start and end
    times are within 10 ms and whose pitch is equal.
    """
    fingering = []
    for line in Path(annotation_path).read_text().splitlines():
        if line.startswith("//") or not line.strip():
            continue
        parts = line.strip().split("\t")
        if len(parts) == 8:
            _, start, end, pitch, _, _, _, finger = parts
            f = int(finger)
            if 0 <= f <= 9:
                fingering.append((float(start), float(end), parse_pitch_to_midi_number(pitch), f))
    seq = parse_midi(midi_path)
    for note in seq.notes:
        for s, e, p, f in fingering:
            if abs(note.start_time - s) < 0.01 and abs(note.end_time - e) < 0.01 and note.pitch == p:
                note.part = f
                break
    return seq


def twinkle_twinkle_little_star_one_hand() -> NoteSequence:
    """``robopianist/music/library.py:69-97``."""
    spec = [(60, 0.0, 0.5, 0), (60, 0.5, 1.0, 0), (67, 1.0, 1.5, 2), (67, 1.5, 2.0, 2),
            (69, 2.0, 2.5, 3), (69, 2.5, 3.0, 3), (67, 3.0, 4.0, 2), (65, 4.0, 4.5, 3),
            (65, 4.5, 5.0, 3), (64, 5.0, 5.5, 2), (64, 5.5, 6.0, 2), (62, 6.0, 6.5, 1),
            (62, 6.5, 7.0, 1), (60, 7.0, 8.0, 0)]
    seq = NoteSequence(title="Twinkle Twinkle (one hand)")
    for p, s, e, f in spec:
        seq.notes.append(Note(p, s, e, 80, f))
    seq.total_time = 8.0
    return seq


# ---------------------------------------------------------------------------------------
# NoteTrajectory.
# ---------------------------------------------------------------------------------------


def note_trajectory(seq: NoteSequence, dt: float):
    """``NoteTrajectory.seq_to_trajectory`` (robopianist/music/midi_file.py:315-362).

    Returns ``notes[T]`` as lists of ``(key, fingering)`` in increasing MIDI pitch order and
    ``sustains[T]``. Frame semantics are those of ``sequence_to_pianoroll``
    (robopianist/music/piano_roll.py:59-204) with ``onset_window=0``: a note occupies
    frames ``[int(s*fps), max(start+1, ceil(e*fps)))``; a note whose onset frame re-strikes
    a key that was active in the previous frame is dropped from that frame.
    """
    fps = 1.0 / dt
    n_frames = int(seq.total_time * fps + 1)
    vel = np.zeros((n_frames, 128), dtype=np.float32)
    onset = np.zeros((n_frames, 128), dtype=np.float32)
    finger = np.full((n_frames, 128), -1, dtype=np.float32)
    cc = np.zeros((n_frames, 128), dtype=np.int32)

    def frames(s, e):
        sf = int(s * fps)
        ef = int(math.ceil(e * fps))
        return sf, max(sf + 1, ef)

    for note in sorted(seq.notes, key=lambda n: n.start_time):
        if note.pitch < 0 or note.pitch > 127:
            continue
        sf, ef = frames(note.start_time, note.end_time)
        onset[sf:min(n_frames, sf + 1), note.pitch] = 1.0
        vel[sf:ef, note.pitch] = note.velocity / MAX_VELOCITY
        finger[sf:ef, note.pitch] = note.part
    for c in seq.control_changes:
        f, _ = frames(c.time, 0)
        if f < n_frames:
            cc[f, c.control_number] = c.control_value + 1
    onset_vel = vel * onset

    notes: List[List[Tuple[int, int]]] = []
    for t in range(n_frames):
        step = []
        for idx in np.nonzero(vel[t])[0]:
            if t > 0 and vel[t - 1][idx] and onset_vel[t][idx]:
                continue
            if not MIN_MIDI_PITCH_PIANO <= idx <= MAX_MIDI_PITCH_PIANO:
                raise ValueError(f"pitch {idx} outside the piano range")
            step.append((int(idx) - MIN_MIDI_PITCH_PIANO, int(finger[t, idx])))
        notes.append(step)
    sustains: List[int] = []
    prev = 0
    for t in range(n_frames):
        ev = cc[t, SUSTAIN_PEDAL_CC_NUMBER]
        if 1 <= ev <= SUSTAIN_PEDAL_CC_NUMBER:
            s = 0
        elif SUSTAIN_PEDAL_CC_NUMBER + 1 <= ev <= MAX_CC_VALUE + 1:
            s = 1
        else:
            s = prev
        sustains.append(s)
        prev = s
    return notes, sustains


@dataclass
class SongTables:
    """Dense per-control-step song tables, the device-side form of a NoteTrajectory.

    ``goal[t, k]`` is 1 for keys active at step t, ``goal[t, 88]`` the sustain target.
    ``keys[t, :count[t]]`` / ``fingers[t, :count[t]]`` hold the step's notes in pitch
    order (fingers 0-4 right hand, 5-9 left hand, -1 unknown).
    """

    name: str
    goal: np.ndarray  # [T, 89] float32
    count: np.ndarray  # [T] int32
    keys: np.ndarray  # [T, MAX_NOTES_PER_STEP] int32
    fingers: np.ndarray  # [T, MAX_NOTES_PER_STEP] int32
    has_fingering: bool

    @property
    def T(self) -> int:
        return int(self.goal.shape[0])


def song_tables(seq: NoteSequence, dt: float, initial_buffer_time: float = 0.0,
                name: Optional[str] = None) -> SongTables:
    """``PianoWithShadowHands._reset_trajectory`` (piano_with_shadow_hands.py:159-165)."""
    notes, sustains = note_trajectory(seq, dt)
    # NoteTrajectory.add_initial_buffer_time (midi_file.py:388-401).
    if initial_buffer_time < 0:
        raise ValueError("initial_buffer_time must be non-negative.")
    nbuf = int(round(initial_buffer_time / dt))
    notes = [[] for _ in range(nbuf)] + notes
    sustains = [0] * nbuf + sustains
    T = len(notes)
    goal = np.zeros((T, NUM_KEYS + 1), dtype=np.float32)
    count = np.zeros(T, dtype=np.int32)
    keys = np.full((T, MAX_NOTES_PER_STEP), -1, dtype=np.int32)
    fingers = np.full((T, MAX_NOTES_PER_STEP), -1, dtype=np.int32)
    for t, step in enumerate(notes):
        if len(step) > MAX_NOTES_PER_STEP:
            raise ValueError(f"step {t} has {len(step)} notes > {MAX_NOTES_PER_STEP}")
        count[t] = len(step)
        for i, (k, f) in enumerate(step):
            goal[t, k] = 1.0
            keys[t, i] = k
            fingers[t, i] = f
        goal[t, NUM_KEYS] = sustains[t]
    return SongTables(name or seq.title, goal, count, keys, fingers, seq.has_fingering())


def test_midi(dt: float = 0.01) -> NoteSequence:
    """``_get_test_midi`` of robopianist/suite/tasks/piano_with_shadow_hands_test.py:29-52."""
    seq = NoteSequence(title="test")
    seq.notes.append(Note(84, 0.0, 2 * dt, 80, 1))  # C6, right index.
    seq.notes.append(Note(79, 2 * dt, 3 * dt, 80, 0))  # G5, right thumb.
    seq.total_time = 3 * dt
    return seq
