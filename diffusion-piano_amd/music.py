"""Song ingestion for the batched piano environment (host precompute, init-time only).

The reference's music pipeline (note_seq / pretty_midi in Python, both absent on the GPU
box) restated natively in ``libpianosong.so`` (``csrc/song.cpp``, C-ABI
``include/pianosong.h``); this module is its Python face and keeps the reference's data
classes:

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
Malformed input raises ``ValueError`` with the library's message.
"""

from __future__ import annotations

import ctypes as C
import re
from dataclasses import dataclass, field
from pathlib import Path
from typing import List, Optional, Tuple

import numpy as np

from . import _lib

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
# libpianosong.so (include/pianosong.h)
# ---------------------------------------------------------------------------------------


class _PssNote(C.Structure):
    _fields_ = [("pitch", C.c_int32), ("start_time", C.c_double), ("end_time", C.c_double),
                ("velocity", C.c_int32), ("part", C.c_int32)]


class _PssCC(C.Structure):
    _fields_ = [("time", C.c_double), ("control_number", C.c_int32), ("control_value", C.c_int32)]


def _check(rc: int) -> None:
    if rc != 0:
        msg = _lib.load_song().pss_last_error()
        raise ValueError(msg.decode() if msg else f"pianosong error {rc}")


class _Seq:
    """Owns a pss_seq handle."""

    def __init__(self, h: C.c_void_p):
        self.h = h

    def __del__(self):
        if getattr(self, "h", None) is not None and self.h.value:
            _lib.load_song().pss_free(self.h)
            self.h = None

    @classmethod
    def parse(cls, data: bytes) -> "_Seq":
        h = C.c_void_p()
        buf = (C.c_uint8 * len(data)).from_buffer_copy(data)
        _check(_lib.load_song().pss_parse_midi(buf, len(data), C.byref(h)))
        return cls(h)

    @classmethod
    def of(cls, seq: NoteSequence) -> "_Seq":
        notes = (_PssNote * max(1, len(seq.notes)))(*[_PssNote(n.pitch, n.start_time, n.end_time, n.velocity, n.part)
                                                      for n in seq.notes])
        ccs = (_PssCC * max(1, len(seq.control_changes)))(
            *[_PssCC(c.time, c.control_number, c.control_value) for c in seq.control_changes])
        h = C.c_void_p()
        _check(_lib.load_song().pss_from_notes(notes, len(seq.notes), ccs, len(seq.control_changes),
                                               float(seq.total_time), C.byref(h)))
        return cls(h)

    def sequence(self, title: str) -> NoteSequence:
        L = _lib.load_song()
        nn, nc, tt = C.c_int(), C.c_int(), C.c_double()
        _check(L.pss_info(self.h, C.byref(nn), C.byref(nc), C.byref(tt), None))
        notes = (_PssNote * max(1, nn.value))()
        ccs = (_PssCC * max(1, nc.value))()
        _check(L.pss_get(self.h, notes, ccs))
        seq = NoteSequence(title=title, total_time=tt.value)
        seq.notes = [Note(n.pitch, n.start_time, n.end_time, n.velocity, n.part) for n in notes[:nn.value]]
        seq.control_changes = [ControlChange(c.time, c.control_number, c.control_value) for c in ccs[:nc.value]]
        return seq


# ---------------------------------------------------------------------------------------
# The reference's functions
# ---------------------------------------------------------------------------------------


def parse_midi(path) -> NoteSequence:
    """Parses a type-0/1 SMF into a :class:`NoteSequence` (``pss_parse_midi``).

    Note pairing follows pretty_midi ``PrettyMIDI._load_instruments``: a note-off (or a
    note-on with velocity 0) closes every open note of that (channel, pitch) that started
    at an earlier tick; an open note started at the same tick stays open. Instruments are
    keyed by (track, channel, program) in first-seen order and their notes are appended
    instrument by instrument, which is the order note_seq copies them into the sequence.
    Ticks map to seconds through the merged tempo map (default 120 qpm).
    """
    return _Seq.parse(Path(path).read_bytes()).sequence(Path(path).stem)


def trim_silence(seq: NoteSequence) -> NoteSequence:
    """``MidiFile.trim_silence``: ``extract_subsequence(seq, notes[0].start, notes[-1].end)``
    (``pss_trim_silence``): notes starting inside ``[start, end)`` shifted by ``-start``, ends
    clipped to ``end``; control changes inside the window shifted; a sustain pedal held at
    ``start`` re-emitted at time 0."""
    s = _Seq.of(seq)
    _check(_lib.load_song().pss_trim_silence(s.h))
    return s.sequence(seq.title)


_NOTE_VALUES = {
    "C": 0, "C#": 1, "Db": 1, "D": 2, "D#": 3, "Eb": 3, "E": 4, "F": 5, "F#": 6,
    "Gb": 6, "G": 7, "G#": 8, "Ab": 8, "A": 9, "A#": 10, "Bb": 10, "B": 11,
}


def parse_pitch_to_midi_number(pitch_str: str) -> int:
    """``data_processing/add_fingering_to_midi.py:7-24``."""
    m = re.match(r"([A-G][#b]?)(\d+)", pitch_str)
    if not m or m.group(1) not in _NOTE_VALUES:
        raise ValueError(f"Invalid pitch format: {pitch_str}")
    note, octave = m.groups()
    return _NOTE_VALUES[note] + (int(octave) + 1) * 12


def add_fingering_from_annotation_file(midi_path, annotation_path) -> NoteSequence:
    """``data_processing/add_fingering_to_midi.py:26-83`` (``pss_add_fingering``).

    Each sequence note takes the finger of the first annotation line whose start and end
    times are within 10 ms and whose pitch is equal.
    """
    s = _Seq.parse(Path(midi_path).read_bytes())
    _check(_lib.load_song().pss_add_fingering(s.h, Path(annotation_path).read_bytes()))
    return s.sequence(Path(midi_path).stem)


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
# NoteTrajectory / device tables.
# ---------------------------------------------------------------------------------------


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


def _tables(seq: NoteSequence, dt: float, initial_buffer_time: float, max_notes: int):
    L = _lib.load_song()
    s = _Seq.of(seq)
    T = C.c_int()
    _check(L.pss_song_tables(s.h, float(dt), float(initial_buffer_time), 0, max_notes, None, None, None, None,
                             C.byref(T)))
    n = T.value
    goal = np.zeros((n, NUM_KEYS + 1), np.float32)
    count = np.zeros(n, np.int32)
    keys = np.full((n, max_notes), -1, np.int32)
    fingers = np.full((n, max_notes), -1, np.int32)
    _check(L.pss_song_tables(s.h, float(dt), float(initial_buffer_time), n, max_notes, goal.ctypes.data,
                             count.ctypes.data, keys.ctypes.data, fingers.ctypes.data, C.byref(T)))
    return goal, count, keys, fingers


def note_trajectory(seq: NoteSequence, dt: float):
    """``NoteTrajectory.seq_to_trajectory`` (robopianist/music/midi_file.py:315-362).

    Returns ``notes[T]`` as lists of ``(key, fingering)`` in increasing MIDI pitch order and
    ``sustains[T]``. Frame semantics are those of ``sequence_to_pianoroll``
    (robopianist/music/piano_roll.py:59-204) with ``onset_window=0``: a note occupies
    frames ``[int(s*fps), max(start+1, ceil(e*fps)))``; a note whose onset frame re-strikes
    a key that was active in the previous frame is dropped from that frame.
    """
    goal, count, keys, fingers = _tables(seq, dt, 0.0, NUM_KEYS)
    notes: List[List[Tuple[int, int]]] = [[(int(keys[t, i]), int(fingers[t, i])) for i in range(count[t])]
                                          for t in range(len(count))]
    return notes, [int(x) for x in goal[:, NUM_KEYS]]


def song_tables(seq: NoteSequence, dt: float, initial_buffer_time: float = 0.0,
                name: Optional[str] = None) -> SongTables:
    """``PianoWithShadowHands._reset_trajectory`` (piano_with_shadow_hands.py:159-165), with
    ``NoteTrajectory.add_initial_buffer_time`` (midi_file.py:388-401)."""
    goal, count, keys, fingers = _tables(seq, dt, initial_buffer_time, MAX_NOTES_PER_STEP)
    return SongTables(name or seq.title, goal, count, keys, fingers, seq.has_fingering())


def test_midi(dt: float = 0.01) -> NoteSequence:
    """``_get_test_midi`` of robopianist/suite/tasks/piano_with_shadow_hands_test.py:29-52."""
    seq = NoteSequence(title="test")
    seq.notes.append(Note(84, 0.0, 2 * dt, 80, 1))  # C6, right index.
    seq.notes.append(Note(79, 2 * dt, 3 * dt, 80, 0))  # G5, right thumb.
    seq.total_time = 3 * dt
    return seq
