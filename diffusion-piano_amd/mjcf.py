"""MJCF-subset loader for user-supplied hand models.

The reference builds each hand with ``mjcf.from_path`` on the Menagerie Shadow Hand XML and
then edits it (robopianist/models/hands/shadow_hand.py:93-311): forearm DOFs with position
actuators and critical damping (``_add_dofs`` :272-311), fingertip sites on the distal
bodies (:181-198), and capsule fingertip colliders under ``primitive_fingertip_collisions``
(:144-152). ``load_hand`` reads such an XML into the ``model.HandSpec`` that
``model.build_model(hand=...)`` compiles. The right hand is read, and the left hand is its
mirror image, as for the authored hand. ``hand_to_mjcf`` writes a HandSpec back out as
Menagerie-style MJCF.

The supported subset is what the hot path simulates:

* ``<compiler angle autolimits eulerseq>``;
* ``<default>`` classes, nested (inheriting) and selected by ``class`` / ``childclass``;
* ``<body pos quat|euler|axisangle|zaxis>`` with ``<inertial pos quat mass diaginertia|fullinertia>``;
* ``<joint type=hinge|slide axis range damping armature>``, and ``stiffness`` must be 0;
* ``<geom>`` colliders (contype or conaffinity non-zero): capsules (``size`` + frame, or
  ``fromto``) and cylinders, which become capsules as in the reference's MJX path
  (parallelized_base.py:49-64); boxes (``size`` = half sizes); meshes, which collide as the
  convex hull of their vertices as in MuJoCo (``<asset><mesh file=... scale=...>`` with an
  OBJ or STL file under ``<compiler meshdir>``, or inline ``vertex=``; the hull is computed
  with qhull, MuJoCo's hull library, and centred at its volume centroid, MuJoCo's mesh
  frame origin; at most ``abi.HULL_MAXVERT`` hull vertices). Non-colliding (visual) geoms
  are skipped; spheres, ellipsoids, planes and primitives fitted to a mesh raise
  ``ValueError``;
* ``<tendon><fixed>`` over two joints;
* ``<actuator><position joint|tendon kp ctrlrange forcerange>``;
* ``<contact><exclude body1 body2>``.

The ABI fixes the hand's sizes (``abi.HAND_NBODY`` bodies, ``HAND_NDOF`` - 2 joints,
``HAND_NACT`` - 2 actuators, ``HAND_NTENDON`` tendons; at most ``HAND_NGEOM`` capsules and
``HAND_NXGEOM`` box / mesh colliders), and a model that differs raises ``ValueError`` naming
the count.
"""

from __future__ import annotations

import math
import xml.etree.ElementTree as ET
from pathlib import Path
from typing import Dict, List, Optional, Tuple, Union

import numpy as np

from . import abi
from . import model as M

# shadow_hand_constants.py:33-40 (order matters: site index = finger index)
FINGERTIP_BODIES = ("thdistal", "ffdistal", "mfdistal", "rfdistal", "lfdistal")
# shadow_hand.py:41-53: the two default forearm DOFs (stiffness = position-actuator kp)
FOREARM_DOFS = (("forearm_tx", 1, (-1.0, 0.0, 0.0), (-1.0, 1.0)),
                ("forearm_ty", 1, (0.0, 0.0, 1.0), M.FOREARM_TY_RANGE))


# ------------------------------------------------------------------ small helpers
def _floats(s: Optional[str]) -> Optional[List[float]]:
    return None if s is None else [float(x) for x in s.split()]


def _qmul(a, b):
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return (w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
            w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2)


def _axis_quat(axis, angle):
    a = np.asarray(axis, np.float64)
    a = a / np.linalg.norm(a)
    s = math.sin(angle / 2)
    return (math.cos(angle / 2), a[0] * s, a[1] * s, a[2] * s)


def _quat_from_z(z):
    """The minimal rotation taking +z to ``z`` (MuJoCo's zaxis / fromto frame)."""
    z = np.asarray(z, np.float64)
    z = z / np.linalg.norm(z)
    c = float(z[2])
    if c > 1.0 - 1e-15:
        return (1.0, 0.0, 0.0, 0.0)
    if c < -1.0 + 1e-15:
        return (0.0, 1.0, 0.0, 0.0)
    axis = np.cross([0.0, 0.0, 1.0], z)
    return _axis_quat(axis, math.acos(c))


class _Ctx:
    def __init__(self, root: ET.Element):
        comp = root.find("compiler")
        get = comp.get if comp is not None else (lambda k, d=None: d)
        self.degree = get("angle", "degree") == "degree"   # MJCF's default unit is degrees
        self.autolimits = get("autolimits", "true") == "true"
        self.eulerseq = get("eulerseq", "xyz")
        self.classes: Dict[str, Dict[str, Dict[str, str]]] = {}
        d = root.find("default")
        if d is not None:
            self._defaults(d, {}, "main")

    def _defaults(self, node, inherited, name):
        own = {tag: dict(attrs) for tag, attrs in inherited.items()}
        for child in node:
            if child.tag != "default":
                own.setdefault(child.tag, {}).update(child.attrib)
        self.classes[name] = own
        for child in node:
            if child.tag == "default":
                cname = child.get("class")
                if not cname:
                    raise ValueError("nested <default> without a class name")
                self._defaults(child, own, cname)

    def attrs(self, el: ET.Element, tag: str, cls: str) -> Dict[str, str]:
        cls = el.get("class", cls)
        if cls not in self.classes and cls != "main":
            raise ValueError(f"<{el.tag}> uses unknown default class {cls!r}")
        out = dict(self.classes.get(cls, {}).get(tag, {}))
        out.update(el.attrib)
        return out

    def angle(self, v: float) -> float:
        return math.radians(v) if self.degree else v

    def frame_quat(self, a: Dict[str, str]):
        if "quat" in a:
            return tuple(_floats(a["quat"]))
        if "axisangle" in a:
            x, y, z, t = _floats(a["axisangle"])
            return _axis_quat((x, y, z), self.angle(t))
        if "euler" in a:
            q = (1.0, 0.0, 0.0, 0.0)
            for ax, t in zip(self.eulerseq, _floats(a["euler"])):
                unit = {"x": (1, 0, 0), "y": (0, 1, 0), "z": (0, 0, 1)}[ax.lower()]
                r = _axis_quat(unit, self.angle(t))
                q = _qmul(q, r) if ax.islower() else _qmul(r, q)   # lower case: rotating axes
            return q
        if "zaxis" in a:
            return _quat_from_z(_floats(a["zaxis"]))
        if "xyaxes" in a:
            v = _floats(a["xyaxes"])
            x = np.asarray(v[:3]) / np.linalg.norm(v[:3])
            y = np.asarray(v[3:]) - x * np.dot(x, v[3:])
            y /= np.linalg.norm(y)
            return _mat_quat(np.stack([x, y, np.cross(x, y)], axis=1))
        return (1.0, 0.0, 0.0, 0.0)

    def limited(self, a: Dict[str, str], flag: str, rng: str) -> bool:
        v = a.get(flag, "auto")
        if v == "auto":
            if not self.autolimits and rng in a:
                raise ValueError(f"{rng} given without {flag} and autolimits is false")
            return rng in a
        return v == "true"


def _mat_quat(R):
    w = math.sqrt(max(0.0, 1.0 + R[0, 0] + R[1, 1] + R[2, 2])) / 2
    if w > 1e-8:
        return (w, (R[2, 1] - R[1, 2]) / (4 * w), (R[0, 2] - R[2, 0]) / (4 * w), (R[1, 0] - R[0, 1]) / (4 * w))
    i = int(np.argmax(np.diag(R)))
    j, k = (i + 1) % 3, (i + 2) % 3
    s = math.sqrt(max(0.0, 1.0 + R[i, i] - R[j, j] - R[k, k])) * 2
    q = [0.0, 0.0, 0.0, 0.0]
    q[0] = (R[k, j] - R[j, k]) / s
    q[1 + i] = s / 4
    q[1 + j] = (R[j, i] + R[i, j]) / s
    q[1 + k] = (R[k, i] + R[i, k]) / s
    return tuple(q)


def _mesh_vertices(path: Path) -> np.ndarray:
    """Vertices of an OBJ (``v`` lines) or STL (binary or ASCII) file."""
    data = path.read_bytes()
    suffix = path.suffix.lower()
    if suffix == ".obj":
        rows = [ln.split()[1:4] for ln in data.decode("utf-8", "replace").splitlines() if ln.startswith("v ")]
        return np.asarray(rows, dtype=np.float64).reshape(-1, 3)
    if suffix == ".stl":
        if data[:5].lower() == b"solid" and b"facet" in data[:2048]:
            rows = [ln.split()[1:4] for ln in data.decode("utf-8", "replace").splitlines()
                    if ln.strip().startswith("vertex")]
            return np.asarray(rows, dtype=np.float64).reshape(-1, 3)
        n = int(np.frombuffer(data[80:84], dtype="<u4")[0])
        rec = np.frombuffer(data[84:84 + 50 * n], dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)),
                                                                  ("a", "<u2")]))
        return rec["v"].reshape(-1, 3).astype(np.float64)
    raise ValueError(f"mesh file {path.name!r}: only .obj and .stl are supported")


def convex_hull_collider(points) -> Tuple[np.ndarray, np.ndarray]:
    """(centre, hull vertices relative to it) of a point set: qhull's convex hull, centred at
    the hull's volume centroid."""
    from scipy.spatial import ConvexHull  # qhull, the library MuJoCo computes mesh hulls with

    pts = np.asarray(points, dtype=np.float64)
    hull = ConvexHull(pts)
    verts = pts[hull.vertices]
    # volume centroid: tetrahedra from an interior point to every facet
    o = verts.mean(axis=0)
    vol, cen = 0.0, np.zeros(3)
    for f in hull.simplices:
        a, b, c = pts[f[0]] - o, pts[f[1]] - o, pts[f[2]] - o
        v = abs(np.dot(a, np.cross(b, c))) / 6.0
        vol += v
        cen += v * (a + b + c) / 4.0
    centre = o + cen / vol
    return centre, verts - centre


def _strip(name: Optional[str], prefix: str) -> Optional[str]:
    if name is not None and prefix and name.startswith(prefix):
        return name[len(prefix):]
    return name


# ------------------------------------------------------------------ fail-closed attribute checks
# The loader must not simulate a different hand than the XML describes: every attribute of the
# elements it reads is either modelled (read into the HandSpec), irrelevant to the dynamics
# (names, visuals, solver effort), or held to the single value the kernel simulates - anything
# else raises ValueError naming the element and attribute.
MJ_SOLREF = (0.02, 1.0)                   # MuJoCo defaults (mjModel solref / solimp / friction)
MJ_SOLIMP = (0.9, 0.95, 0.001, 0.5, 2.0)
MJ_FRICTION = 1.0

_VISUAL = {"name", "class", "group", "rgba", "material", "user"}
_FRAME = {"pos", "quat", "euler", "axisangle", "zaxis", "xyaxes"}
_ALLOWED = {
    "body": _VISUAL | _FRAME | {"childclass"},
    "inertial": _FRAME | {"mass", "diaginertia", "fullinertia"},
    "joint": _VISUAL | {"type", "axis", "range", "limited", "damping", "armature", "frictionloss", "springref"},
    "geom": _VISUAL | _FRAME | {"type", "size", "fromto", "mesh", "contype", "conaffinity", "friction", "solref",
                                "solimp", "density", "mass", "shellinertia", "fluidshape", "fluidcoef"},
    "position": _VISUAL | {"joint", "tendon", "kp", "ctrlrange", "ctrllimited", "forcerange", "forcelimited"},
    "fixed": _VISUAL | {"limited", "solreflimit", "solimplimit", "range"},
    "option": {"timestep", "iterations", "ls_iterations", "tolerance", "ls_tolerance", "solver", "jacobian",
               "noslip_tolerance", "ccd_iterations", "ccd_tolerance", "sdf_iterations", "sdf_initpoints",
               "apirate"},
    "compiler": {"angle", "autolimits", "eulerseq", "meshdir", "assetdir", "texturedir", "discardvisual",
                 "strippath", "usethread", "inertiagrouprange", "exactmeshinertia", "saveinertial"},
}
# attribute -> (the one value the kernel simulates, parser)
_NUM = lambda v: tuple(float(x) for x in v.split())
_FIXED = {
    "body": {"mocap": ("false", str), "gravcomp": ((0.0,), _NUM)},
    "joint": {"pos": ((0.0, 0.0, 0.0), _NUM), "ref": ((0.0,), _NUM), "stiffness": ((0.0,), _NUM),
              "margin": ((0.0,), _NUM), "solreflimit": (MJ_SOLREF, _NUM), "solimplimit": (MJ_SOLIMP, _NUM),
              "solreffriction": (MJ_SOLREF, _NUM), "solimpfriction": (MJ_SOLIMP, _NUM),
              "actuatorfrclimited": ("false", str), "actuatorgravcomp": ("false", str)},
    "geom": {"condim": ((3.0,), _NUM), "margin": ((0.0,), _NUM), "gap": ((0.0,), _NUM),
             "priority": ((0.0,), _NUM), "solmix": ((1.0,), _NUM)},
    "position": {"kv": ((0.0,), _NUM), "gear": ((1.0,), _NUM), "dampratio": ((0.0,), _NUM),
                 "timeconst": ((0.0,), _NUM), "inheritrange": ((0.0,), _NUM), "actlimited": ("false", str),
                 "actearly": ("false", str)},
    "fixed": {"stiffness": ((0.0,), _NUM), "damping": ((0.0,), _NUM), "frictionloss": ((0.0,), _NUM),
              "margin": ((0.0,), _NUM), "springlength": ((-1.0, -1.0), _NUM)},
    "option": {"integrator": ("Euler", str), "cone": ("pyramidal", str), "impratio": ((1.0,), _NUM),
               "noslip_iterations": ((0.0,), _NUM), "gravity": ((0.0, 0.0, -9.81), _NUM),
               "wind": ((0.0, 0.0, 0.0), _NUM), "density": ((0.0,), _NUM), "viscosity": ((0.0,), _NUM),
               "o_margin": ((0.0,), _NUM)},
    "compiler": {"inertiafromgeom": ("false|auto", str), "balanceinertia": ("false", str),
                 "boundmass": ((0.0,), _NUM), "boundinertia": ((0.0,), _NUM), "settotalmass": ((-1.0,), _NUM),
                 "fusestatic": ("false", str), "coordinate": ("local", str), "alignfree": ("false", str)},
}


def _pad(vals, full):
    """MuJoCo fills a partial solref / solimp / friction from its defaults."""
    return tuple(vals) + tuple(full[len(vals):])


def check_attrs(kind: str, what: str, a: Dict[str, str]) -> None:
    """Raise ValueError if ``a`` (an element's attributes with its class defaults merged) holds an
    attribute the kernel does not simulate, or a held attribute at another value."""
    allowed, fixed = _ALLOWED[kind], _FIXED.get(kind, {})
    for k, v in a.items():
        if k in allowed:
            continue
        if k not in fixed:
            raise ValueError(f"{what}: attribute {k}={v!r} is not supported (the kernel does not model it)")
        want, parse = fixed[k]
        if parse is str:
            ok = v in want.split("|")
        else:
            try:
                got = parse(v)
            except ValueError:
                raise ValueError(f"{what}: bad {k}={v!r}") from None
            ok = len(got) <= len(want) and np.allclose(_pad(got, want), want, rtol=0, atol=1e-12)
        if not ok:
            raise ValueError(f"{what}: {k}={v!r} is not supported (the kernel simulates {k}={want!r})")


_TOP = {"compiler", "option", "size", "default", "asset", "worldbody", "contact", "tendon", "actuator", "sensor",
        "keyframe", "visual", "statistic", "custom"}
_BODY_CHILDREN = {"inertial", "joint", "geom", "body", "site", "camera", "light"}


# ------------------------------------------------------------------ loader
def load_hand(source: Union[str, Path], prefix: str = "rh_") -> M.HandSpec:
    """Read a right-hand MJCF (a path, or the XML text itself) into a ``model.HandSpec``,
    with the reference's forearm DOFs and fingertip sites added (shadow_hand.py:181-198,
    272-311). ``prefix`` is stripped from element names (Menagerie's ``rh_``)."""
    text = source if isinstance(source, str) and source.lstrip().startswith("<") else Path(source).read_text()
    root = ET.fromstring(text)
    if root.tag != "mujoco":
        raise ValueError("not an MJCF document (root element is not <mujoco>)")
    for el in root:
        if el.tag not in _TOP:
            raise ValueError(f"<{el.tag}> is not supported (the kernel does not model it)")
    for opt in root.findall("option"):
        check_attrs("option", "<option>", dict(opt.attrib))
        for fl in opt:
            raise ValueError(f"<option><{fl.tag} {' '.join(f'{k}={v!r}' for k, v in fl.attrib.items())}> "
                             "is not supported (the kernel runs MuJoCo's default flags)")
    for comp_el in root.findall("compiler"):
        check_attrs("compiler", "<compiler>", dict(comp_el.attrib))
    for cel in root.findall("contact"):
        for el in cel:
            if el.tag != "exclude":
                raise ValueError(f"<contact><{el.tag}> is not supported (only <exclude>)")
    for tel in root.findall("tendon"):
        for el in tel:
            if el.tag != "fixed":
                raise ValueError(f"<tendon><{el.tag}> is not supported (only two-joint <fixed>)")
    ctx = _Ctx(root)
    base_dir = Path(source).parent if not (isinstance(source, str) and source.lstrip().startswith("<")) else Path(".")
    comp = root.find("compiler")
    mesh_dir = base_dir / (comp.get("meshdir", comp.get("assetdir", "")) if comp is not None else "")
    meshes: Dict[str, ET.Element] = {}
    for asset in root.findall("asset"):
        for me in asset.findall("mesh"):
            mname = me.get("name") or Path(me.get("file", "")).stem
            meshes[mname] = me

    def mesh_points(mname: str) -> np.ndarray:
        me = meshes.get(mname)
        if me is None:
            raise ValueError(f"unknown mesh {mname!r}")
        if me.get("vertex"):
            pts = np.asarray(_floats(me.get("vertex")), dtype=np.float64).reshape(-1, 3)
        elif me.get("file"):
            pts = _mesh_vertices(mesh_dir / me.get("file"))
        else:
            raise ValueError(f"mesh {mname!r} has neither file= nor vertex=")
        return pts * np.asarray(_floats(me.get("scale", "1 1 1")), dtype=np.float64)

    wb = root.find("worldbody")
    roots = [] if wb is None else wb.findall("body")
    if len(roots) != 1:
        raise ValueError(f"expected one hand root body under <worldbody>, found {len(roots)}")

    bodies: List[M.Body] = []
    dofs: List[M.Dof] = []
    geoms: List[M.Geom] = []
    xgeoms: List[M.XGeom] = []
    body_idx: Dict[str, int] = {}
    joint_idx: Dict[str, int] = {}
    root_joint_attrs: Dict[str, str] = {}
    contact_params = set()

    def visit(el: ET.Element, parent: int, cls: str):
        cls = el.get("childclass", cls)
        a = ctx.attrs(el, "body", cls)
        bi = len(bodies)
        name = _strip(a.get("name", f"body{bi}"), prefix)
        check_attrs("body", f"body {name!r}", {k: v for k, v in el.attrib.items()})
        for child in el:
            if child.tag not in _BODY_CHILDREN:
                raise ValueError(f"body {name!r}: <{child.tag}> is not supported")
        body_idx[name] = bi
        pos = tuple(_floats(a.get("pos", "0 0 0")))
        quat = ctx.frame_quat(a)
        mass, ipos, iquat, diag = 0.0, (0.0, 0.0, 0.0), (1.0, 0.0, 0.0, 0.0), (0.0, 0.0, 0.0)
        inertial = el.find("inertial")
        if inertial is not None:
            ia = ctx.attrs(inertial, "inertial", cls)
            check_attrs("inertial", f"body {name!r} <inertial>", ia)
            mass = float(ia["mass"])
            ipos = tuple(_floats(ia.get("pos", "0 0 0")))
            if "diaginertia" in ia:
                iquat = ctx.frame_quat(ia)
                diag = tuple(_floats(ia["diaginertia"]))
            elif "fullinertia" in ia:
                xx, yy, zz, xy, xz, yz = _floats(ia["fullinertia"])
                w, V = np.linalg.eigh(np.array([[xx, xy, xz], [xy, yy, yz], [xz, yz, zz]]))
                if np.linalg.det(V) < 0:
                    V[:, 0] = -V[:, 0]
                iquat, diag = _mat_quat(V), tuple(float(x) for x in w)
            else:
                raise ValueError(f"body {name!r}: <inertial> needs diaginertia or fullinertia")
        elif parent >= 0:
            raise ValueError(f"body {name!r}: no <inertial> (inertia from geoms is not supported)")
        bodies.append(M.Body(name, parent, pos, quat, mass, ipos, iquat, diag))
        for j in el.findall("joint"):
            ja = ctx.attrs(j, "joint", cls)
            if float(ja.get("stiffness", "0")) != 0.0:
                raise ValueError(f"joint {ja.get('name')!r}: joint stiffness is not supported")
            check_attrs("joint", f"joint {ja.get('name')!r}", ja)
            if bi == 0:
                root_joint_attrs.update(ja)
            jtype = ja.get("type", "hinge")
            if jtype not in ("hinge", "slide"):
                raise ValueError(f"joint {ja.get('name')!r}: type {jtype!r} is not supported (hinge/slide)")
            if float(ja.get("stiffness", "0")) != 0.0:
                raise ValueError(f"joint {ja.get('name')!r}: joint stiffness is not supported")
            kind = 0 if jtype == "hinge" else 1
            rng = (0.0, 0.0)
            if ctx.limited(ja, "limited", "range"):
                lo, hi = _floats(ja["range"])
                rng = (ctx.angle(lo), ctx.angle(hi)) if kind == 0 else (lo, hi)
            else:
                raise ValueError(f"joint {ja.get('name')!r}: unlimited joints are not supported")
            jname = _strip(ja.get("name", f"joint{len(dofs)}"), prefix)
            joint_idx[jname] = len(dofs)
            dofs.append(M.Dof(jname, bi, kind, tuple(_floats(ja.get("axis", "0 0 1"))), rng,
                              float(ja.get("damping", "0")), float(ja.get("armature", "0")),
                              float(ja.get("frictionloss", "0"))))
        for g in el.findall("geom"):
            ga = ctx.attrs(g, "geom", cls)
            if int(ga.get("contype", "1")) == 0 and int(ga.get("conaffinity", "1")) == 0:
                continue  # visual only
            check_attrs("geom", f"body {name!r} collider", ga)
            for bit in ("contype", "conaffinity"):
                if ga.get(bit, "1") not in ("0", "1"):
                    raise ValueError(f"body {name!r} collider: {bit}={ga[bit]!r} is not supported (bitmask "
                                     "filtering is not modelled: 0 or 1)")
            if ga.get("contype", "1") != "1" or ga.get("conaffinity", "1") != "1":
                raise ValueError(f"body {name!r} collider: contype/conaffinity other than 1/1 is not supported")
            param = (_pad(_floats(ga.get("solref", "")) or (), MJ_SOLREF),
                     _pad(_floats(ga.get("solimp", "")) or (), MJ_SOLIMP),
                     (_floats(ga.get("friction", "")) or [MJ_FRICTION])[0])
            contact_params.add(param)
            gtype = ga.get("type", "sphere")
            if gtype not in ("capsule", "cylinder", "box", "mesh"):
                raise ValueError(f"body {name!r}: collider type {gtype!r} is not supported "
                                 "(capsule/cylinder, box, mesh)")
            if gtype != "mesh" and "mesh" in ga:
                raise ValueError(f"body {name!r}: a {gtype} fitted to mesh {ga['mesh']!r} is not supported")
            size = _floats(ga.get("size", "0"))
            if gtype == "box":
                if len(size) < 3:
                    raise ValueError(f"body {name!r}: box needs size='x y z' half sizes")
                xgeoms.append(M.XGeom(bi, "box", tuple(_floats(ga.get("pos", "0 0 0"))),
                                      tuple(ctx.frame_quat(ga)), tuple(size[:3])))
                continue
            if gtype == "mesh":
                if "mesh" not in ga:
                    raise ValueError(f"body {name!r}: mesh geom without mesh=")
                centre, verts = convex_hull_collider(mesh_points(ga["mesh"]))
                if len(verts) > abi.HULL_MAXVERT:
                    raise ValueError(f"mesh {ga['mesh']!r}: convex hull has {len(verts)} vertices; "
                                     f"at most {abi.HULL_MAXVERT} are supported")
                q = M.quat_normalize(ctx.frame_quat(ga))
                gpos = np.asarray(_floats(ga.get("pos", "0 0 0"))) + M.quat_to_mat(q) @ centre
                xgeoms.append(M.XGeom(bi, "hull", tuple(gpos), tuple(q), verts=verts))
                continue
            if "fromto" in ga:
                ft = np.asarray(_floats(ga["fromto"]), np.float64)
                p0, p1 = ft[:3], ft[3:]
                d = p1 - p0
                half = float(np.linalg.norm(d)) / 2
                gpos, axis = tuple((p0 + p1) / 2), tuple(d / (2 * half))
            else:
                if len(size) < 2:
                    raise ValueError(f"body {name!r}: capsule needs size='radius half-length'")
                half = size[1]
                gpos = tuple(_floats(ga.get("pos", "0 0 0")))
                axis = tuple(M.quat_to_mat(M.quat_normalize(ctx.frame_quat(ga)))[:, 2])
            geoms.append(M.Geom(bi, gpos, axis, half, size[0]))
        for child in el.findall("body"):
            visit(child, bi, cls)

    visit(roots[0], -1, "main")
    n_menagerie_joints = len(dofs)

    # forearm DOFs on the root body after its own joints (shadow_hand.py:272-311); they
    # take the root's joint defaults (armature), damping is set by build_model (critical)
    ra = ctx.attrs(roots[0].find("joint") if roots[0].find("joint") is not None else ET.Element("joint"),
                   "joint", roots[0].get("childclass", "main"))
    arm, floss = float(ra.get("armature", "0")), float(ra.get("frictionloss", "0"))
    n_root = sum(1 for d in dofs if d.body == 0)
    slides = [M.Dof(n, 0, k, ax, rng, 0.0, arm, floss) for (n, k, ax, rng) in FOREARM_DOFS]
    dofs[n_root:n_root] = slides
    remap = [i if i < n_root else i + len(slides) for i in range(n_menagerie_joints)]
    joint_idx = {k: remap[v] for k, v in joint_idx.items()}

    tendons: List[Tuple[int, int]] = []
    tcoef: List[Tuple[float, float]] = []
    tendon_idx: Dict[str, int] = {}
    tel = root.find("tendon")
    for t in ([] if tel is None else tel.findall("fixed")):
        check_attrs("fixed", f"fixed tendon {t.get('name')!r}", ctx.attrs(t, "fixed", "main"))
        if t.get("limited", "auto") == "true" or (t.get("limited", "auto") == "auto" and "range" in t.attrib):
            raise ValueError(f"fixed tendon {t.get('name')!r}: tendon limits are not supported")
        js = t.findall("joint")
        if len(js) != 2:
            raise ValueError(f"fixed tendon {t.get('name')!r}: exactly two joints are supported")
        try:
            pair = tuple(joint_idx[_strip(j.get("joint"), prefix)] for j in js)
        except KeyError as e:
            raise ValueError(f"fixed tendon {t.get('name')!r}: unknown joint {e}") from None
        tendon_idx[_strip(t.get("name", f"tendon{len(tendons)}"), prefix)] = len(tendons)
        tendons.append(pair)
        tcoef.append(tuple(float(j.get("coef", "1")) for j in js))

    acts = []
    ael = root.find("actuator")
    for a in ([] if ael is None else list(ael)):
        if a.tag != "position":
            raise ValueError(f"actuator <{a.tag}> is not supported (position only)")
        aa = ctx.attrs(a, "position", "main")
        check_attrs("position", f"actuator {aa.get('name')!r}", aa)
        if "joint" in aa:
            kind, target = 0, joint_idx.get(_strip(aa["joint"], prefix))
        elif "tendon" in aa:
            kind, target = 1, tendon_idx.get(_strip(aa["tendon"], prefix))
        else:
            raise ValueError(f"actuator {aa.get('name')!r}: needs joint= or tendon=")
        if target is None:
            raise ValueError(f"actuator {aa.get('name')!r}: unknown target")
        if not ctx.limited(aa, "ctrllimited", "ctrlrange"):
            raise ValueError(f"actuator {aa.get('name')!r}: ctrlrange is required")
        cr = tuple(_floats(aa["ctrlrange"]))
        fr = tuple(_floats(aa["forcerange"])) if ctx.limited(aa, "forcelimited", "forcerange") else None
        acts.append((kind, target, float(aa.get("kp", "1")), cr, fr))
    for (n, _, _, rng) in FOREARM_DOFS:
        acts.append((0, joint_idx.setdefault(n, [d.name for d in dofs].index(n)), M.FOREARM_KP, rng, None))

    excludes = []
    cel = root.find("contact")
    for e in ([] if cel is None else cel.findall("exclude")):
        try:
            excludes.append((body_idx[_strip(e.get("body1"), prefix)], body_idx[_strip(e.get("body2"), prefix)]))
        except KeyError as err:
            raise ValueError(f"<exclude>: unknown body {err}") from None

    sites = []
    for b in FINGERTIP_BODIES:
        if b not in body_idx:
            raise ValueError(f"fingertip body {prefix + b!r} not found")
        sites.append((body_idx[b], (0.0, 0.0, M.THUMBTIP_OFFSET if b == "thdistal" else M.FINGERTIP_OFFSET)))

    # joints_pos observation order: the model's joints in document order, forearm ones last
    obs_order = [remap[i] for i in range(n_menagerie_joints)] + [n_root + i for i in range(len(slides))]

    for what, got, want in (("bodies", len(bodies), abi.HAND_NBODY), ("joints", len(dofs), abi.HAND_NDOF),
                            ("actuators", len(acts), abi.HAND_NACT), ("fixed tendons", len(tendons), abi.HAND_NTENDON)):
        if got != want:
            raise ValueError(f"hand has {got} {what} (with the forearm DOFs); the kernel ABI needs {want}")
    for what, got, most in (("capsule/cylinder colliders", len(geoms), abi.HAND_NGEOM),
                            ("box/mesh colliders", len(xgeoms), abi.HAND_NXGEOM)):
        if got > most:
            raise ValueError(f"hand has {got} {what}; the kernel ABI holds at most {most}")
    if len(contact_params) > 1:
        raise ValueError(f"hand colliders carry {len(contact_params)} different solref/solimp/friction sets; the "
                         "kernel's hand contact parameters are one set (ps_model_desc.hand_contact)")
    contact = next(iter(contact_params)) if contact_params else (MJ_SOLREF, MJ_SOLIMP, MJ_FRICTION)
    return M.HandSpec(bodies, dofs, geoms, excludes, sites, tendons, acts, obs_order, tcoef, xgeoms or None,
                      contact)


# ------------------------------------------------------------------ writer
def _fmt(v) -> str:
    return " ".join(repr(float(x)) for x in v)


def hand_to_mjcf(spec: M.HandSpec, prefix: str = "rh_") -> str:
    """Menagerie-style MJCF of a HandSpec, without its forearm DOFs (``load_hand`` adds them
    back, as the reference's ``_add_dofs`` does). Joint defaults go through nested classes,
    finger colliders are written as ``fromto`` capsules and each body gets a visual geom, so
    that the loader's class, frame and filtering paths are all exercised on a round trip."""
    root = ET.Element("mujoco", model="right_shadow_hand")
    ET.SubElement(root, "compiler", angle="radian", autolimits="true")
    dflt = ET.SubElement(root, "default")
    hand = ET.SubElement(dflt, "default", {"class": "right_hand"})
    floss = spec.dofs[2].frictionloss
    ET.SubElement(hand, "joint", axis="1 0 0", damping="0.05", armature=repr(spec.dofs[2].armature),
                  frictionloss=repr(float(floss)))
    ET.SubElement(hand, "position", forcerange="-1 1")
    wrist = ET.SubElement(hand, "default", {"class": "wrist"})
    ET.SubElement(wrist, "joint", damping="0.5")
    sr, si, fr = spec.contact or (MJ_SOLREF, MJ_SOLIMP, MJ_FRICTION)
    ET.SubElement(ET.SubElement(hand, "default", {"class": "plastic_collision"}), "geom", type="capsule",
                  group="3", solref=_fmt(sr), solimp=_fmt(si), friction=_fmt((fr, 0.005, 0.0001)))
    ET.SubElement(ET.SubElement(hand, "default", {"class": "plastic_visual"}), "geom", type="mesh",
                  contype="0", conaffinity="0", group="2")

    if spec.xgeoms:
        assets = ET.SubElement(root, "asset")
        for j, xg in enumerate(spec.xgeoms):
            if xg.kind == "hull":
                ET.SubElement(assets, "mesh", name=f"hull{j}", vertex=_fmt(np.asarray(xg.verts).ravel()))
    names = {i: b.name for i, b in enumerate(spec.bodies)}
    els: Dict[int, ET.Element] = {}
    wb = ET.SubElement(root, "worldbody")
    slide_names = {n for (n, _, _, _) in FOREARM_DOFS}
    for i, b in enumerate(spec.bodies):
        parent = wb if b.parent < 0 else els[b.parent]
        attrs = {"name": prefix + b.name, "pos": _fmt(b.pos), "quat": _fmt(b.quat)}
        if b.parent < 0:
            attrs["childclass"] = "right_hand"
        el = ET.SubElement(parent, "body", attrs)
        els[i] = el
        ET.SubElement(el, "inertial", pos=_fmt(b.ipos), quat=_fmt(b.iquat), mass=repr(b.mass),
                      diaginertia=_fmt(b.diag))
        for d in spec.dofs:
            if d.body != i or d.name in slide_names:
                continue
            ja = {"name": prefix + d.name, "range": _fmt(d.range)}
            if d.kind == 1:
                ja["type"] = "slide"
            if d.name.startswith("WRJ"):
                ja["class"] = "wrist"
                if d.damping != 0.5:
                    ja["damping"] = repr(d.damping)
            elif d.damping != 0.05:
                ja["damping"] = repr(d.damping)
            if tuple(d.axis) != (1.0, 0.0, 0.0):
                ja["axis"] = _fmt(d.axis)
            if d.armature != spec.dofs[2].armature:
                ja["armature"] = repr(d.armature)
            if d.frictionloss != floss:
                ja["frictionloss"] = repr(float(d.frictionloss))
            ET.SubElement(el, "joint", ja)
        ET.SubElement(el, "geom", {"class": "plastic_visual", "mesh": b.name})
        for g in spec.geoms:
            if g.body != i:
                continue
            if b.name.endswith(("proximal", "middle", "distal")) and not b.name.startswith("th"):
                p, a = np.asarray(g.pos), np.asarray(g.axis) * g.halflen
                ET.SubElement(el, "geom", {"class": "plastic_collision", "size": repr(g.radius),
                                           "fromto": _fmt(np.concatenate([p - a, p + a]))})
            else:
                ET.SubElement(el, "geom", {"class": "plastic_collision", "size": _fmt((g.radius, g.halflen)),
                                           "pos": _fmt(g.pos), "quat": _fmt(_quat_from_z(g.axis))})
        for j, xg in enumerate(spec.xgeoms or []):
            if xg.body != i:
                continue
            if xg.kind == "box":
                ET.SubElement(el, "geom", {"class": "plastic_collision", "type": "box", "size": _fmt(xg.size),
                                           "pos": _fmt(xg.pos), "quat": _fmt(xg.quat)})
            else:
                ET.SubElement(el, "geom", {"class": "plastic_collision", "type": "mesh", "mesh": f"hull{j}",
                                           "pos": _fmt(xg.pos), "quat": _fmt(xg.quat)})
    cont = ET.SubElement(root, "contact")
    for a, b in spec.excludes:
        ET.SubElement(cont, "exclude", body1=prefix + names[a], body2=prefix + names[b])
    ten = ET.SubElement(root, "tendon")
    coefs = spec.tendon_coef or [(1.0, 1.0)] * len(spec.tendons)
    for t, (d2, d1) in enumerate(spec.tendons):
        fe = ET.SubElement(ten, "fixed", name=f"{prefix}T{t}")
        for d, c in ((d2, coefs[t][0]), (d1, coefs[t][1])):
            ET.SubElement(fe, "joint", joint=prefix + spec.dofs[d].name, coef=repr(c))
    act = ET.SubElement(root, "actuator")
    for (kind, target, kp, cr, fr) in spec.acts:
        if kind == 0 and spec.dofs[target].name in slide_names:
            continue
        aa = {"class": "right_hand", "kp": repr(kp), "ctrlrange": _fmt(cr)}
        if kind == 0:
            aa["joint"] = prefix + spec.dofs[target].name
        else:
            aa["tendon"] = f"{prefix}T{target}"
        if fr is None:
            aa["forcelimited"] = "false"
        elif tuple(fr) != (-1.0, 1.0):
            aa["forcerange"] = _fmt(fr)
        ET.SubElement(act, "position", aa)
    ET.indent(root)
    return ET.tostring(root, encoding="unicode")


def capsule_points(radius, halflen, n_ring=8, n_lat=2) -> np.ndarray:
    """Points on a capsule surface along z (a rounded fingertip shape for hull colliders)."""
    pts = []
    for z0, sgn in ((halflen, 1.0), (-halflen, -1.0)):
        pts.append((0.0, 0.0, z0 + sgn * radius))
        for j in range(n_lat + 1):
            phi = (j / (n_lat + 1)) * np.pi / 2  # 0 at the equator
            for i in range(n_ring):
                t = 2 * np.pi * (i + 0.5 * (j % 2)) / n_ring
                pts.append((radius * np.cos(phi) * np.cos(t), radius * np.cos(phi) * np.sin(t),
                            z0 + sgn * radius * np.sin(phi)))
    return np.asarray(pts)


def box_hull_hand(hull_fingertips: bool = True) -> M.HandSpec:
    """The authored right hand with the reference's collider kinds (shadow_hand.py:95,144-152:
    Menagerie palm boxes and distal meshes): the two palm capsules and the little-finger
    metacarpal capsule become boxes, and with ``hull_fingertips`` (the reference's default
    ``primitive_fingertip_collisions=False``) every distal capsule a 58-point capsule-shaped convex
    hull (MuJoCo collides a mesh as its hull); without, the distal colliders stay capsules (the
    reference's ``primitive_fingertip_collisions=True`` turns its distal meshes into capsules).
    ``TaskConfig(primitive_fingertip_collisions=...)`` selects it, as does
    ``TaskConfig(hand_xml=hand_to_mjcf(box_hull_hand()))`` through the MJCF path; the step kernel's
    box / hull instantiation (pianosim_kernel<true>) then runs."""
    hand = M.authored_hand()
    geoms, xgeoms = [], []
    names = [b.name for b in hand.bodies]
    for g in hand.geoms:
        bname = names[g.body]
        if bname == "palm" or bname == "lfmetacarpal":
            q = _quat_from_z(g.axis)
            xgeoms.append(M.XGeom(g.body, "box", tuple(g.pos), tuple(q), (g.radius, g.radius * 0.8, g.halflen + g.radius)))
        elif bname.endswith("distal") and hull_fingertips:
            c, v = convex_hull_collider(capsule_points(g.radius, g.halflen))
            R = M.quat_to_mat(_quat_from_z(g.axis))
            pos = np.asarray(g.pos) + R @ c
            xgeoms.append(M.XGeom(g.body, "hull", tuple(pos), tuple(_quat_from_z(g.axis)), verts=v))
        else:
            geoms.append(g)
    return hand._replace(geoms=geoms, xgeoms=xgeoms)
