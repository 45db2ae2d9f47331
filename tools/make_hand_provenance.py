"""Writes diffusion-piano_amd/hand_provenance.json: every quantity of the authored right hand
(model.authored_hand()) with its public source, so that dropping in the real Menagerie file
(mjcf.load_hand) is a mechanical diff. Run once after an intentional
change of the authored hand; tests/test_hand_provenance.py checks the hand against the file.

Sources:
* MJX  = MuJoCo Menagerie shadow_hand/right_hand.xml (Shadow Hand E3M5), the file the
  reference copies in (scripts/install_deps.sh:81 pins Menagerie 1afc8be; the file is NOT in
  this container, the values were transcribed from the public model and are unverified here);
* RP   = the reference's own edits (robopianist/models/hands/shadow_hand.py,
  robopianist/suite/tasks/base.py), verifiable here;
* DEV  = a documented deviation of this implementation.
"""
import importlib
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

MJX = "Menagerie shadow_hand/right_hand.xml"
CLASS = {  # joint -> Menagerie default class that sets its axis / range / actuator
    "WRJ2": "wrist_y", "WRJ1": "wrist_x", "THJ5": "thbase", "THJ4": "thproximal", "THJ3": "thhub",
    "THJ2": "thmiddle", "THJ1": "thdistal", "LFJ5": "metacarpal",
}


def jclass(name):
    if name in CLASS:
        return CLASS[name]
    return {"4": "knuckle", "3": "proximal", "2": "middle_distal", "1": "middle_distal"}[name[-1]]


def table():
    """The provenance table of model.authored_hand() as a JSON-ready dict."""
    model = importlib.import_module("diffusion-piano_amd.model")
    hand = model.authored_hand()
    rows = []

    def add(q, value, source, status):
        rows.append({"quantity": q, "value": value, "source": source, "status": status})

    for i, b in enumerate(hand.bodies):
        nm = "rh_" + b.name
        if i == 0:
            add(f"body {nm} pos", list(b.pos), "RP tasks/base.py:34-37 (attachment frame replaces the root pose)",
                "verifiable")
        else:
            add(f"body {nm} pos", list(b.pos), f"{MJX} <body name='{nm}' pos>", "transcribed")
            add(f"body {nm} quat", list(b.quat), f"{MJX} <body name='{nm}' quat>", "transcribed")
        add(f"body {nm} parent", b.parent, f"{MJX} body nesting", "transcribed")
        add(f"body {nm} mass", b.mass, f"{MJX} <body name='{nm}'><inertial mass>", "transcribed")
        add(f"body {nm} ipos", list(b.ipos), f"{MJX} <inertial pos>", "transcribed")
        add(f"body {nm} iquat", list(b.iquat), f"{MJX} <inertial quat>", "transcribed")
        add(f"body {nm} diaginertia", list(b.diag), f"{MJX} <inertial diaginertia>", "transcribed")
    for d in hand.dofs:
        if d.name.startswith("forearm"):
            src = "RP shadow_hand.py:41-52 _FOREARM_DOFS (axis, range); range of forearm_tx reset by tasks/base.py:160-194"
            add(f"joint {d.name} axis", list(d.axis), src, "verifiable")
            add(f"joint {d.name} range", list(d.range), src, "verifiable")
            add(f"joint {d.name} damping", d.damping,
                "RP shadow_hand.py:299-301 critical damping 2 sqrt(m_subtree kp), set in model.build_model",
                "verifiable")
        else:
            c = jclass(d.name)
            add(f"joint rh_{d.name} axis", list(d.axis), f"{MJX} <default class='{c}'><joint axis> (else class right_hand 1 0 0)",
                "transcribed")
            add(f"joint rh_{d.name} range", list(d.range), f"{MJX} <default class='{c}'><joint range>", "transcribed")
            add(f"joint rh_{d.name} damping", d.damping,
                f"{MJX} <default class='{'wrist' if d.name.startswith('WR') else 'right_hand'}'><joint damping>",
                "transcribed")
        add(f"joint {d.name} armature", d.armature, f"{MJX} <default class='right_hand'><joint armature>", "transcribed")
        add(f"joint {d.name} frictionloss", d.frictionloss,
            f"{MJX} <default class='right_hand'><joint frictionloss> (the forearm slides inherit the root "
            "childclass, shadow_hand.py:272-311); one friction-loss row per dof in every substep's solve",
            "transcribed")
    dof_names = [d.name for d in hand.dofs]
    for a, (kind, target, kp, cr, fr) in enumerate(hand.acts):
        tname = dof_names[target] if kind == 0 else f"tendon {target}"
        if kind == 0 and dof_names[target].startswith("forearm"):
            src = "RP shadow_hand.py:41-52,303-309 (position actuator, kp = stiffness 300, ctrlrange = joint range)"
            status = "verifiable"
        else:
            src = f"{MJX} <actuator><position class=...> of {tname} (kp, ctrlrange, forcerange)"
            status = "transcribed"
        add(f"actuator {a} ({tname}) kind", kind, src, status)
        add(f"actuator {a} ({tname}) kp", kp, src, status)
        add(f"actuator {a} ({tname}) ctrlrange", list(cr), src, status)
        add(f"actuator {a} ({tname}) forcerange", None if fr is None else list(fr), src, status)
    for t, (d2, d1) in enumerate(hand.tendons):
        add(f"tendon {t} joints", [dof_names[d2], dof_names[d1]], f"{MJX} <tendon><fixed name='rh_*J0'> joints *J2 + *J1",
            "transcribed")
    for g, geom in enumerate(hand.geoms):
        add(f"collider {g} (body {hand.bodies[geom.body].name}) capsule",
            {"pos": list(geom.pos), "axis": list(geom.axis), "halflen": geom.halflen, "radius": geom.radius},
            "DEV: authored capsule standing in for the Menagerie collision geom(s) of this body "
            "(boxes on forearm/palm, capsules on phalanges, mesh fingertips by default: shadow_hand.py:95,144-152)",
            "deviation")
    for s, (body, pos) in enumerate(hand.sites):
        add(f"fingertip site {s} ({hand.bodies[body].name})", list(pos),
            "RP shadow_hand.py:81-82,190-207 (_FINGERTIP_OFFSET 0.026, _THUMBTIP_OFFSET 0.0275 along the distal z)",
            "verifiable")
    for a, b in hand.excludes:
        add("contact exclude", [hand.bodies[a].name, hand.bodies[b].name], f"{MJX} <contact><exclude>", "transcribed")
    sr, si, fr = hand.contact
    src = f"{MJX} <default class='plastic'>/<geom> contact attributes of the collision geoms"
    add("collider solref", list(sr), src, "transcribed")
    add("collider solimp", list(si), src, "transcribed")
    add("collider friction (sliding)", fr, src, "transcribed")
    assumed = ("ASSUMED: MuJoCo's default (the Menagerie XML is not in this container); mjcf.load_hand raises "
               "on any other value in a user XML")
    add("collider condim", 3, assumed, "assumed")
    add("collider margin / gap", [0.0, 0.0], assumed, "assumed")
    add("collider contype / conaffinity", [1, 1], assumed, "assumed")
    add("joint solreffriction", [0.02, 1.0], assumed, "assumed")
    add("joint solimpfriction", [0.9, 0.95, 0.001, 0.5, 2.0], assumed, "assumed")
    add("joint solreflimit", [0.02, 1.0], assumed, "assumed")
    add("joint solimplimit", [0.9, 0.95, 0.001, 0.5, 2.0], assumed, "assumed")
    add("option integrator", "Euler", assumed + " (dm_control composer physics; the reference sets none)", "assumed")
    add("option cone", "pyramidal", assumed, "assumed")
    add("option impratio", 1.0, assumed, "assumed")
    add("option noslip_iterations", 0, assumed, "assumed")
    add("joints_pos order", [dof_names[i] for i in hand.obs_order],
        "RP hands/base.py:76-78 + shadow_hand_test.py:101-106 (Menagerie joints, forearm joints appended)", "verifiable")
    out = {"hand": "Shadow Hand E3M5 (right; the left hand is its mirror image, model.build_model)",
           "sources": {"MJX": MJX + " at Menagerie 1afc8be (scripts/install_deps.sh:81); absent from this container",
                       "RP": "reference files under /root/reference/robopianist",
                       "DEV": "deviation, DESIGN.md section 3",
                       "ASSUMED": "a MuJoCo default the absent XML may override; the loader fails closed on it"},
           "counts": {"bodies": len(hand.bodies), "dofs": len(hand.dofs), "actuators": len(hand.acts),
                      "tendons": len(hand.tendons), "colliders": len(hand.geoms), "sites": len(hand.sites)},
           "rows": rows}
    return out


def main():
    out = table()
    rows = out["rows"]
    path = ROOT / "diffusion-piano_amd" / "hand_provenance.json"
    path.write_text(json.dumps(out, indent=1) + "\n")
    print(f"{len(rows)} rows -> {path}")


if __name__ == "__main__":
    main()
