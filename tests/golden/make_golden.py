"""Generate the golden fixtures under tests/golden/ from the reference's own code.

Runs only in the build container (it reads /root/reference, which does not exist on the
GPU box). The reference's music code imports note_seq / pretty_midi / dm_control, none of
which are installed, so small stub modules are registered first; the reference source
files are then loaded by path and executed unmodified:

* robopianist/music/{constants,piano_roll,midi_file,library}.py  -> song trajectories
  (NoteTrajectory.seq_to_trajectory, the Twinkle song itself from library.py).
* robopianist/models/piano/{piano_constants,piano_mjcf}.py -> piano key geometry, with a
  recording stand-in for dm_control.mjcf.RootElement.
* scipy.optimize.linear_sum_assignment (the reference's OT-fingering dependency, present
  here) -> assignment known answers.

What is NOT pinned by this script: the SMF parse of the two .mid files and the
trim_silence window (note_seq is absent); those inputs are produced by this repo's
parser (``music.parse_midi`` / ``music.trim_silence``) and the reference trajectory code
is run on them. The fixtures record which input path was used.

Usage: python tests/golden/make_golden.py  (writes tests/golden/*.json)
"""

from __future__ import annotations

import importlib.util
import json
import sys
import types
from pathlib import Path

import numpy as np

REF = Path("/root/reference")
ROOT = Path(__file__).resolve().parents[2]
OUT = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT))
import importlib  # noqa: E402

our_music = importlib.import_module("diffusion-piano_amd.music")  # only for the .mid parse, see docstring


# --------------------------------------------------------------------------- stubs
class _Rep(list):
    def __init__(self, factory):
        super().__init__()
        self._factory = factory

    def add(self, **kw):
        obj = self._factory(**kw)
        self.append(obj)
        return obj


class _Obj(types.SimpleNamespace):
    pass


def _note(**kw):
    d = dict(pitch=0, start_time=0.0, end_time=0.0, velocity=0, part=0, instrument=0)
    d.update(kw)
    return _Obj(**d)


def _cc(**kw):
    d = dict(time=0.0, control_number=0, control_value=0, instrument=0)
    d.update(kw)
    return _Obj(**d)


class NoteSequence:
    def __init__(self):
        self.notes = _Rep(_note)
        self.control_changes = _Rep(_cc)
        self.tempos = _Rep(lambda **kw: _Obj(**kw))
        self.sequence_metadata = _Obj(title="", artist="")
        self.total_time = 0.0


def _install_stubs():
    note_seq = types.ModuleType("note_seq")
    consts = types.ModuleType("note_seq.constants")
    consts.MIN_MIDI_VELOCITY = 0
    consts.MAX_MIDI_VELOCITY = 127
    consts.DEFAULT_QUARTERS_PER_MINUTE = 120.0
    consts.MIN_MIDI_PITCH = 0
    consts.MAX_MIDI_PITCH = 127
    consts.STANDARD_PPQ = 220
    pb2 = types.ModuleType("note_seq.protobuf.music_pb2")
    pb2.NoteSequence = NoteSequence
    proto = types.ModuleType("note_seq.protobuf")
    proto.music_pb2 = pb2
    note_seq.constants = consts
    note_seq.music_pb2 = pb2
    note_seq.protobuf = proto
    note_seq.NoteSequence = NoteSequence
    for name in ("midi_io", "midi_synth", "sequences_lib"):
        m = types.ModuleType("note_seq." + name)
        setattr(note_seq, name, m)
        sys.modules["note_seq." + name] = m
    sys.modules.update({
        "note_seq": note_seq, "note_seq.constants": consts,
        "note_seq.protobuf": proto, "note_seq.protobuf.music_pb2": pb2,
        "pretty_midi": types.ModuleType("pretty_midi"),
    })
    rp = types.ModuleType("robopianist")
    rp.__path__ = []
    rp.SF2_PATH = "/nonexistent.sf2"
    rpm = types.ModuleType("robopianist.music")
    rpm.__path__ = []
    audio = types.ModuleType("robopianist.music.audio")
    sys.modules.update({"robopianist": rp, "robopianist.music": rpm,
                        "robopianist.music.audio": audio})
    rpm.audio = audio


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    parent, _, child = name.rpartition(".")
    if parent in sys.modules:
        setattr(sys.modules[parent], child, mod)
    return mod


def _to_ref_seq(seq):
    """Our parsed NoteSequence -> stub protobuf NoteSequence."""
    out = NoteSequence()
    for n in seq.notes:
        out.notes.add(pitch=n.pitch, start_time=n.start_time, end_time=n.end_time,
                      velocity=n.velocity, part=n.part)
    for c in seq.control_changes:
        out.control_changes.add(time=c.time, control_number=c.control_number,
                                control_value=c.control_value)
    out.total_time = seq.total_time
    return out


def _traj_record(midi_file_mod, seq, dt, source):
    notes, sustains = midi_file_mod.NoteTrajectory.seq_to_trajectory(seq, dt)
    return {
        "source": source,
        "dt": dt,
        "T": len(notes),
        "notes": [[[int(n.key), int(n.fingering)] for n in step] for step in notes],
        "sustains": [int(s) for s in sustains],
        "has_fingering": bool(midi_file_mod.MidiFile(seq=seq).has_fingering()),
    }


def songs():
    mconst = _load("robopianist.music.constants", REF / "robopianist/music/constants.py")
    assert mconst.NUM_KEYS == 88
    _load("robopianist.music.piano_roll", REF / "robopianist/music/piano_roll.py")
    mf = _load("robopianist.music.midi_file", REF / "robopianist/music/midi_file.py")
    lib = _load("robopianist.music.library", REF / "robopianist/music/library.py")

    rec = {}
    twinkle = lib.twinkle_twinkle_little_star_one_hand().seq
    rec["twinkle"] = _traj_record(mf, twinkle, 0.05, "reference library.py:69-97")

    # Reference test MIDIs (midi_file_test.py:109-177, piano_with_shadow_hands_test.py:29-52).
    seq = NoteSequence()
    seq.notes.add(start_time=0.01, end_time=0.02, velocity=80, pitch=84, part=-1)
    seq.notes.add(start_time=0.02, end_time=0.05, velocity=80, pitch=84, part=-1)
    seq.total_time = 0.05
    rec["test_restrike"] = _traj_record(mf, seq, 0.01, "midi_file_test.py:109-131")
    seq = NoteSequence()
    seq.notes.add(start_time=0.0, end_time=0.01, velocity=80, pitch=84, part=-1)
    seq.control_changes.add(time=0.0, control_number=64, control_value=64)
    seq.control_changes.add(time=0.03, control_number=64, control_value=0)
    seq.notes.add(start_time=0.05, end_time=0.06, velocity=80, pitch=84, part=-1)
    seq.total_time = 0.06
    rec["test_sustain"] = _traj_record(mf, seq, 0.01, "midi_file_test.py:134-170")
    seq = NoteSequence()
    seq.notes.add(start_time=0.0, end_time=0.02, velocity=80, pitch=84, part=1)
    seq.notes.add(start_time=0.02, end_time=0.03, velocity=80, pitch=79, part=0)
    seq.total_time = 0.03
    rec["test_task"] = _traj_record(mf, seq, 0.01, "piano_with_shadow_hands_test.py:29-52")

    cf_path = REF / "midi_files_cut/Crossing Field Cut 10s.mid"
    cf = our_music.trim_silence(our_music.parse_midi(cf_path))
    rec["crossing_field"] = _traj_record(
        mf, _to_ref_seq(cf), 0.05, "repo SMF parse + trim_silence -> reference seq_to_trajectory")
    gu = our_music.add_fingering_from_annotation_file(
        REF / "midi_files_cut/Guren no Yumiya Cut 14s.mid",
        REF / "data_processing/Guren no Yumiya Cut 14s_fingering v3.txt")
    gu = our_music.trim_silence(gu)
    rec["guren"] = _traj_record(
        mf, _to_ref_seq(gu), 0.05,
        "repo SMF parse + fingering match + trim_silence -> reference seq_to_trajectory")
    return rec


# --------------------------------------------------------------------------- piano
class _Elem:
    def __init__(self, tag, **kw):
        self.tag = tag
        self.attrs = dict(kw)
        self.children = []

    def add(self, tag, **kw):
        e = _Elem(tag, **kw)
        self.children.append(e)
        return e

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        e = self.__dict__.setdefault("_sub_" + name, _Elem(name))
        return e

    def __setattr__(self, name, value):
        if name in ("tag", "attrs", "children") or name.startswith("_sub_"):
            object.__setattr__(self, name, value)
        else:
            self.attrs[name] = value


def piano():
    dmc = types.ModuleType("dm_control")
    mjcf = types.ModuleType("dm_control.mjcf")
    mjcf.RootElement = lambda: _Elem("mujoco")
    dmc.mjcf = mjcf
    mu = types.ModuleType("mujoco_utils")
    mu.types = types.ModuleType("mujoco_utils.types")
    mu.types.MjcfRootElement = object
    sys.modules.update({"dm_control": dmc, "dm_control.mjcf": mjcf, "mujoco_utils": mu,
                        "mujoco_utils.types": mu.types})
    rpm = types.ModuleType("robopianist.models")
    rpm.__path__ = []
    rpp = types.ModuleType("robopianist.models.piano")
    rpp.__path__ = []
    sys.modules.update({"robopianist.models": rpm, "robopianist.models.piano": rpp})
    pc = _load("robopianist.models.piano.piano_constants",
               REF / "robopianist/models/piano/piano_constants.py")
    pm = _load("robopianist.models.piano.piano_mjcf", REF / "robopianist/models/piano/piano_mjcf.py")
    root = pm.build()
    defaults = {}
    for d in root.default.children:
        defaults[d.attrs["dclass"]] = {
            "geom_size": list(d.geom.attrs["size"]), "mass": d.geom.attrs["mass"],
            "joint_pos": list(d.joint.attrs["pos"]), "damping": d.joint.attrs["damping"],
            "armature": d.joint.attrs["armature"], "stiffness": d.joint.attrs["stiffness"],
            "springref": d.joint.attrs["springref"], "range": list(d.joint.attrs["range"]),
        }
    bodies = [c for c in root.worldbody.children if c.tag == "body"]
    base = bodies[0]
    keys = []
    for b in bodies[1:]:
        geom = b.children[0]
        keys.append({"name": b.attrs["name"], "pos": list(b.attrs["pos"]),
                     "dclass": geom.attrs["dclass"]})
    return {
        "source": "reference piano_mjcf.build() (piano_mjcf.py:25-402), stubbed mjcf",
        "base_pos": list(base.attrs["pos"]),
        "base_size": list(base.children[0].attrs["size"]),
        "defaults": defaults,
        "keys": keys,
        "piano_length": pc.PIANO_LENGTH,
    }


def lsa():
    from scipy.optimize import linear_sum_assignment
    rng = np.random.RandomState(0)
    cases = []
    for k in [1, 2, 3, 5, 8, 10, 12]:
        for _ in range(4):
            c = rng.uniform(0, 0.5, size=(10, k))
            r, col = linear_sum_assignment(c)
            cases.append({"cost": c.tolist(), "rows": r.tolist(), "cols": col.tolist()})
    return {"source": "scipy.optimize.linear_sum_assignment (scipy 1.15.3)", "cases": cases}


def main():
    _install_stubs()
    OUT.mkdir(parents=True, exist_ok=True)
    (OUT / "songs.json").write_text(json.dumps(songs()))
    (OUT / "piano.json").write_text(json.dumps(piano(), indent=1))
    (OUT / "lsa.json").write_text(json.dumps(lsa()))
    print("wrote", sorted(p.name for p in OUT.glob("*.json")))


if __name__ == "__main__":
    main()
