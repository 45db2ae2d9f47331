"""Host precompute and oracle primitives against the reference's golden vectors."""
import numpy as np
import pytest

from helpers import DATA, song


@pytest.mark.parametrize("name", ["twinkle", "crossing_field", "guren", "test_task"])
def test_song_tables_match_reference_trajectory(dp, golden, name):
    g = golden["songs"][name]
    seq = song(dp, name)
    if name in ("crossing_field", "guren"):
        seq = dp.music.trim_silence(seq)
    st = dp.music.song_tables(seq, g["dt"])
    assert st.T == g["T"]
    assert st.has_fingering == g["has_fingering"]
    for t in range(st.T):
        want = g["notes"][t]
        got = [[int(st.keys[t, i]), int(st.fingers[t, i])] for i in range(st.count[t])]
        assert got == want, (name, t)
        goal = np.zeros(89, np.float32)
        for k, _ in want:
            goal[k] = 1
        goal[88] = g["sustains"][t]
        np.testing.assert_array_equal(st.goal[t], goal)


@pytest.mark.parametrize("name", ["test_restrike", "test_sustain"])
def test_reference_trajectory_known_answers(dp, golden, name):
    """midi_file_test.py:179-211: re-strike leaves an empty frame; CC64 sustain."""
    g = golden["songs"][name]
    m = dp.music
    seq = m.NoteSequence()
    if name == "test_restrike":
        seq.notes = [m.Note(84, 0.01, 0.02, 80, -1), m.Note(84, 0.02, 0.05, 80, -1)]
        seq.total_time = 0.05
    else:
        seq.notes = [m.Note(84, 0.0, 0.01, 80, -1), m.Note(84, 0.05, 0.06, 80, -1)]
        seq.control_changes = [m.ControlChange(0.0, 64, 64), m.ControlChange(0.03, 64, 0)]
        seq.total_time = 0.06
    notes, sustains = m.note_trajectory(seq, 0.01)
    assert [[list(x) for x in step] for step in notes] == g["notes"]
    assert sustains == g["sustains"]
    if name == "test_restrike":
        assert len(notes) == 6 and notes[2] == [] and len(notes[3]) == 1
    else:
        assert len(notes) == 7 and sustains[:3] == [1, 1, 1] and sustains[3:6] == [0, 0, 0]


def test_guren_fingering_matches_every_note(dp):
    seq = song(dp, "guren")
    assert len(seq.notes) == 214
    annotated = set()
    for line in (DATA / "Guren no Yumiya Cut 14s_fingering v3.txt").read_text().splitlines():
        parts = line.split("\t")
        if len(parts) == 8:
            annotated.add((float(parts[1]), dp.music.parse_pitch_to_midi_number(parts[3])))
    hits = sum(1 for n in seq.notes if any(abs(n.start_time - s) < 0.01 and n.pitch == p for s, p in annotated))
    assert hits == 214
    assert seq.has_fingering()


def test_crossing_field_has_no_fingering(dp):
    seq = song(dp, "crossing_field")
    assert len(seq.notes) == 18 and not seq.has_fingering()


def test_piano_model_matches_reference_build(dp, golden):
    p = golden["piano"]
    md = dp.model.build_model()
    for k, key in enumerate(p["keys"]):
        np.testing.assert_allclose(list(md.key_pos[k]), key["pos"], atol=1e-12)
        d = p["defaults"][key["dclass"]]
        np.testing.assert_allclose(np.array(list(md.key_half[k])), d["geom_size"], atol=1e-12)
        assert md.key_mass[k] == d["mass"]
        np.testing.assert_allclose(list(md.key_anchor[k]), d["joint_pos"], atol=1e-12)
        assert md.key_damping[k] == d["damping"] and md.key_armature[k] == d["armature"]
        assert md.key_stiffness[k] == d["stiffness"]
        np.testing.assert_allclose(md.key_springref[k], d["springref"])
        np.testing.assert_allclose(list(md.key_range[k]), d["range"])
    np.testing.assert_allclose(list(md.base_pos), p["base_pos"])
    np.testing.assert_allclose(list(md.base_half), p["base_size"])
    # keys sorted along y (broadphase assumption)
    y = [md.key_pos[k][1] for k in range(88)]
    assert all(a < b for a, b in zip(y, y[1:]))


def test_tolerance_known_answers(ref):
    """dm_control rewards.tolerance, gaussian, value_at_margin=0.1."""
    assert ref.tolerance(1.0, 0, 0.05, 0.5) == pytest.approx(2.4547089e-4, rel=1e-6)
    assert ref.tolerance(-1.0, 0, 0.05, 0.5) == pytest.approx(1e-4, rel=1e-6)
    assert ref.tolerance(0.05, 0, 0.01, 0.1) == pytest.approx(0.69183097, rel=1e-6)
    assert ref.tolerance(0.02, 0, 0.05, 0.5) == 1.0
    # key_press at rest with a goal key and no wrong press: 0.5*tol(1) + 0.5
    assert 0.5 * ref.tolerance(1.0, 0, 0.05, 0.5) + 0.5 == pytest.approx(0.50012274, rel=1e-7)


def test_assignment_matches_scipy(ref, golden):
    for case in golden["lsa"]["cases"]:
        c = np.array(case["cost"])
        want = sum(ref.tolerance(c[r, k], 0, 0.01, 0.1) for r, k in zip(case["rows"], case["cols"]))
        if c.shape[1] <= 10:
            got = ref.assignment_tol(c.T)
        else:
            got = ref.assignment_tol(c)
        assert got == pytest.approx(want, rel=1e-9, abs=1e-12)
        # optimal cost identical
