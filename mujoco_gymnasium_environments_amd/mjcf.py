"""MJCF -> struct-of-arrays model compiler (host side, fp64).

Replaces the model-construction half of the reference's MuJoCo boundary:
``mujoco.MjModel.from_xml_string`` (e.g. humanoid_soccer_env/soccer_env.py:80) and the
name tables behind ``mujoco.mj_name2id`` / ``mj_id2name`` (soccer_env.py:222-263, :797).

The seven reference tasks use a small MJCF subset: primitive
geoms only (plane, sphere, capsule, box, cylinder), hinge/slide/free joints, motor and
position actuators, explicit <pair>s, one top-level <default> (plus optional classes).
This compiler implements that subset with MuJoCo's documented compile semantics
[ext, MuJoCo "Modeling"/"XML reference" chapters]:

* depth-first body numbering in XML order, geoms numbered body by body;
* joint/dof address tables, ``qpos0`` (free joint = body pose), ``qpos_spring``;
* ``inertiafromgeom`` (exact capsule inertia with hemispheres), ``mass=`` overrides,
  principal axes of composite bodies;
* ``fromto``, ``quat``/``euler``/``axisangle``/``xyaxes``/``zaxis``, ``angle=degree|radian``;
* ``<freejoint>`` ignores joint defaults (armature/damping/stiffness = 0);
* weld ids, parent/child collision filtering, contype/conaffinity, pair parameter mixing
  (condim/friction max, margin/gap max, solref/solimp mixed by solmix);
* ``mj_setConst``-style constants at qpos0: body/dof ``invweight0`` and ``meaninertia``.

The output is a :class:`Model` of numpy arrays named after mjModel fields; ``Model.pack()``
turns it into the C struct declared in ``include/mgx.h``.
"""
from __future__ import annotations

import math
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

# geom types (mjtGeom order: the narrowphase table is indexed type1 <= type2)
GEOM_PLANE, GEOM_HFIELD, GEOM_SPHERE, GEOM_CAPSULE, GEOM_ELLIPSOID, GEOM_CYLINDER, GEOM_BOX = range(7)
GEOM_TYPES = {"plane": 0, "hfield": 1, "sphere": 2, "capsule": 3, "ellipsoid": 4, "cylinder": 5, "box": 6}
# joint types (mjtJoint)
JNT_FREE, JNT_BALL, JNT_SLIDE, JNT_HINGE = range(4)
JNT_TYPES = {"free": 0, "ball": 1, "slide": 2, "hinge": 3}
# solvers / integrators / cones (mjtSolver, mjtIntegrator, mjtCone)
SOLVERS = {"pgs": 0, "cg": 1, "newton": 2}
INTEGRATORS = {"euler": 0, "rk4": 1, "implicit": 2, "implicitfast": 3}
CONES = {"pyramidal": 0, "elliptic": 1}
MINVAL = 1e-15


def _floats(s: Optional[str], n: Optional[int] = None, default=None):
    if s is None:
        return None if default is None else np.array(default, dtype=np.float64)
    v = np.array([float(x) for x in s.split()], dtype=np.float64)
    if n is not None and v.size < n:
        v = np.concatenate([v, np.zeros(n - v.size)])
    return v


# ---------------------------------------------------------------------------------------
# small quaternion helpers (w, x, y, z), fp64
# ---------------------------------------------------------------------------------------
def quat_mul(a, b):
    return np.array([
        a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
        a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
        a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
        a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]])


def quat_normalize(q):
    n = np.linalg.norm(q)
    return np.array([1.0, 0, 0, 0]) if n < MINVAL else q / n


def quat2mat(q):
    w, x, y, z = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def mat2quat(R):
    t = np.trace(R)
    if t > 0:
        s = math.sqrt(t + 1.0) * 2
        q = [0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s]
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = math.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        q = [(R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s]
    elif R[1, 1] > R[2, 2]:
        s = math.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        q = [(R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s]
    else:
        s = math.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
        q = [(R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s]
    q = np.array(q)
    if q[0] < 0:
        q = -q
    return quat_normalize(q)


def axis_angle_quat(axis, angle):
    axis = np.asarray(axis, dtype=np.float64)
    n = np.linalg.norm(axis)
    if n < MINVAL or angle == 0:
        return np.array([1.0, 0, 0, 0])
    axis = axis / n
    s = math.sin(angle / 2)
    return np.array([math.cos(angle / 2), axis[0] * s, axis[1] * s, axis[2] * s])


def quat_z2vec(vec):
    """Quaternion rotating (0,0,1) onto vec (mju_quatZ2Vec semantics)."""
    v = np.asarray(vec, dtype=np.float64)
    n = np.linalg.norm(v)
    if n < MINVAL:
        return np.array([1.0, 0, 0, 0])
    v = v / n
    z = np.array([0.0, 0, 1])
    a = np.cross(z, v)
    s = np.linalg.norm(a)
    if s < MINVAL:
        return np.array([1.0, 0, 0, 0]) if v[2] > 0 else np.array([0.0, 1, 0, 0])
    a /= s
    ang = math.atan2(s, float(np.dot(z, v)))
    return axis_angle_quat(a, ang)


# ---------------------------------------------------------------------------------------
# default classes
# ---------------------------------------------------------------------------------------
class _Defaults:
    """MJCF <default> tree: class name -> {element tag -> attribute dict}."""

    def __init__(self):
        self.classes: Dict[str, Dict[str, Dict[str, str]]] = {"main": {}}
        self.parent: Dict[str, Optional[str]] = {"main": None}

    def load(self, elem: ET.Element, name: str = "main", parent: Optional[str] = None):
        if name not in self.classes:
            self.classes[name] = {}
            self.parent[name] = parent
        for child in elem:
            if child.tag == "default":
                self.load(child, child.get("class", name), name)
            else:
                self.classes[name].setdefault(child.tag, {}).update(child.attrib)

    def attrs(self, cls: str, tag: str) -> Dict[str, str]:
        chain = []
        c: Optional[str] = cls if cls in self.classes else "main"
        while c is not None:
            chain.append(c)
            c = self.parent[c]
        out: Dict[str, str] = {}
        for c in reversed(chain):
            out.update(self.classes[c].get(tag, {}))
            # actuator shortcuts inherit from <general> defaults too
        return out


@dataclass
class Model:
    """Compiled model: numpy arrays named after mjModel fields (fp64 / int32)."""
    name: str = ""
    # options
    timestep: float = 0.002
    gravity: np.ndarray = field(default_factory=lambda: np.array([0, 0, -9.81]))
    iterations: int = 100
    tolerance: float = 1e-8
    ls_iterations: int = 50
    solver: int = 2
    integrator: int = 0
    cone: int = 0
    impratio: float = 1.0
    meaninertia: float = 1.0
    # sizes
    nq: int = 0
    nv: int = 0
    nu: int = 0
    nbody: int = 0
    njnt: int = 0
    ngeom: int = 0
    nM: int = 0
    # names
    body_names: List[str] = field(default_factory=list)
    jnt_names: List[str] = field(default_factory=list)
    geom_names: List[str] = field(default_factory=list)
    actuator_names: List[str] = field(default_factory=list)
    site_names: List[str] = field(default_factory=list)
    arrays: Dict[str, np.ndarray] = field(default_factory=dict)

    def __getattr__(self, k):
        arrays = self.__dict__.get("arrays")
        if arrays is not None and k in arrays:
            return arrays[k]
        raise AttributeError(k)

    def name2id(self, objtype: str, name: str) -> int:
        """mujoco.mj_name2id restated: -1 when absent (soccer_env.py:236-240 relies on it)."""
        table = {"body": self.body_names, "joint": self.jnt_names, "geom": self.geom_names,
                 "actuator": self.actuator_names, "site": self.site_names}[objtype]
        try:
            return table.index(name)
        except ValueError:
            return -1

    def id2name(self, objtype: str, i: int) -> Optional[str]:
        table = {"body": self.body_names, "joint": self.jnt_names, "geom": self.geom_names,
                 "actuator": self.actuator_names, "site": self.site_names}[objtype]
        if 0 <= i < len(table):
            return table[i] or None
        return None


# ---------------------------------------------------------------------------------------
# compiler
# ---------------------------------------------------------------------------------------
def _geom_mass_inertia(gtype, size, density):
    """Volume-based mass and principal inertia of a primitive (MuJoCo mjCGeom::SetInertia)."""
    if gtype == GEOM_SPHERE:
        r = size[0]
        vol = 4.0 / 3.0 * math.pi * r ** 3
        m = density * vol
        I = 2.0 / 5.0 * m * r * r
        return m, np.array([I, I, I])
    if gtype == GEOM_CAPSULE:
        r, h = size[0], 2 * size[1]
        vol = math.pi * r * r * h + 4.0 / 3.0 * math.pi * r ** 3
        m = density * vol
        ms = m * 4 * r / (4 * r + 3 * h)
        mc = m - ms
        Ix = mc * (3 * r * r + h * h) / 12.0
        Iz = mc * r * r / 2.0
        si = 2 * ms * r * r / 5.0
        Ix += si + ms * h * (3 * r + 2 * h) / 8.0
        Iz += si
        return m, np.array([Ix, Ix, Iz])
    if gtype == GEOM_CYLINDER:
        r, h = size[0], 2 * size[1]
        m = density * math.pi * r * r * h
        Ix = m * (3 * r * r + h * h) / 12.0
        return m, np.array([Ix, Ix, m * r * r / 2.0])
    if gtype == GEOM_BOX:
        a, b, c = size[0], size[1], size[2]
        m = density * 8 * a * b * c
        return m, np.array([m * (b * b + c * c) / 3.0, m * (a * a + c * c) / 3.0, m * (a * a + b * b) / 3.0])
    if gtype == GEOM_ELLIPSOID:
        a, b, c = size[0], size[1], size[2]
        m = density * 4.0 / 3.0 * math.pi * a * b * c
        return m, np.array([m * (b * b + c * c) / 5.0, m * (a * a + c * c) / 5.0, m * (a * a + b * b) / 5.0])
    return 0.0, np.zeros(3)   # plane / hfield: no mass


def _rbound(gtype, size):
    if gtype == GEOM_SPHERE:
        return size[0]
    if gtype == GEOM_CAPSULE:
        return size[0] + size[1]
    if gtype == GEOM_CYLINDER:
        return math.sqrt(size[0] ** 2 + size[1] ** 2)
    if gtype in (GEOM_BOX, GEOM_ELLIPSOID):
        return float(np.linalg.norm(size[:3])) if gtype == GEOM_BOX else float(max(size[:3]))
    return 0.0


class _Compiler:
    def __init__(self, xml: str):
        self.root = ET.fromstring(xml)
        self.defaults = _Defaults()
        comp = self.root.find("compiler")
        self.degree = True   # MuJoCo default angle unit
        self.inertiafromgeom = "auto"
        self.eulerseq = "xyz"
        self.autolimits = True
        if comp is not None:
            self.degree = comp.get("angle", "degree") == "degree"
            self.inertiafromgeom = comp.get("inertiafromgeom", "auto")
            self.eulerseq = comp.get("eulerseq", "xyz")
            self.autolimits = comp.get("autolimits", "true") == "true"
        for d in self.root.findall("default"):
            self.defaults.load(d)

    # --- attribute resolution with defaults ---
    def _attrs(self, elem: ET.Element, cls: str, tag: Optional[str] = None) -> Dict[str, str]:
        c = elem.get("class", cls)
        a = dict(self.defaults.attrs(c, tag or elem.tag))
        a.update(elem.attrib)
        return a

    def _angle(self, v: float) -> float:
        return v * math.pi / 180.0 if self.degree else v

    def _orient(self, a: Dict[str, str]) -> np.ndarray:
        if "quat" in a:
            return quat_normalize(_floats(a["quat"], 4))
        if "axisangle" in a:
            v = _floats(a["axisangle"], 4)
            return axis_angle_quat(v[:3], self._angle(v[3]))
        if "euler" in a:
            e = [self._angle(x) for x in _floats(a["euler"], 3)]
            q = np.array([1.0, 0, 0, 0])
            for ch, ang in zip(self.eulerseq, e):
                ax = {"x": [1, 0, 0], "y": [0, 1, 0], "z": [0, 0, 1]}[ch.lower()]
                r = axis_angle_quat(ax, ang)
                q = quat_mul(q, r) if ch.islower() else quat_mul(r, q)
            return quat_normalize(q)
        if "xyaxes" in a:
            v = _floats(a["xyaxes"], 6)
            x = v[:3] / np.linalg.norm(v[:3])
            y = v[3:] - np.dot(v[3:], x) * x
            y /= np.linalg.norm(y)
            z = np.cross(x, y)
            return mat2quat(np.stack([x, y, z], axis=1))
        if "zaxis" in a:
            return quat_z2vec(_floats(a["zaxis"], 3))
        return np.array([1.0, 0, 0, 0])

    def compile(self, name: str = "") -> Model:
        m = Model(name=name or self.root.get("model", ""))
        opt = self.root.find("option")
        if opt is not None:
            m.timestep = float(opt.get("timestep", m.timestep))
            m.iterations = int(opt.get("iterations", m.iterations))
            m.ls_iterations = int(opt.get("ls_iterations", m.ls_iterations))
            m.tolerance = float(opt.get("tolerance", m.tolerance))
            m.solver = SOLVERS[opt.get("solver", "Newton").lower()]
            m.integrator = INTEGRATORS[opt.get("integrator", "Euler").lower()]
            m.cone = CONES[opt.get("cone", "pyramidal").lower()]
            m.impratio = float(opt.get("impratio", 1.0))
            if "gravity" in opt.attrib:
                m.gravity = _floats(opt.get("gravity"), 3)

        bodies: List[dict] = []
        joints: List[dict] = []
        geoms: List[dict] = []
        sites: List[dict] = []

        def walk(elem: ET.Element, parent: int, cls: str):
            bid = len(bodies)
            a = self._attrs(elem, cls, "body") if bid else {}
            b = dict(name=elem.get("name", "" if bid else "world"), parent=parent,
                     pos=_floats(a.get("pos"), 3, [0, 0, 0]) if bid else np.zeros(3),
                     quat=self._orient(a) if bid else np.array([1.0, 0, 0, 0]),
                     joints=[], geoms=[], inertial=None, mocap=a.get("mocap") == "true")
            bodies.append(b)
            childcls = elem.get("childclass", cls)
            for ch in elem:
                if ch.tag in ("joint", "freejoint"):
                    ja = self._attrs(ch, childcls, "joint") if ch.tag == "joint" else dict(ch.attrib)
                    jt = JNT_FREE if ch.tag == "freejoint" else JNT_TYPES[ja.get("type", "hinge")]
                    if ch.tag == "freejoint":
                        ja = {"name": ch.get("name", "")}
                    j = dict(name=ja.get("name", ""), type=jt, body=bid,
                             pos=_floats(ja.get("pos"), 3, [0, 0, 0]),
                             axis=_floats(ja.get("axis"), 3, [0, 0, 1]),
                             damping=float(ja.get("damping", 0)), armature=float(ja.get("armature", 0)),
                             stiffness=float(ja.get("stiffness", 0)),
                             frictionloss=float(ja.get("frictionloss", 0)),
                             margin=float(ja.get("margin", 0)),
                             ref=float(ja.get("ref", 0)), springref=float(ja.get("springref", 0)),
                             solref=_floats(ja.get("solreflimit"), 2, [0.02, 1.0]),
                             solimp=_floats(ja.get("solimplimit"), 5, [0.9, 0.95, 0.001, 0.5, 2.0]))
                    rng = _floats(ja.get("range"), 2, [0, 0])
                    lim = ja.get("limited", "auto")
                    limited = (lim == "true") or (lim == "auto" and self.autolimits and "range" in ja)
                    if jt == JNT_HINGE:
                        rng = np.array([self._angle(rng[0]), self._angle(rng[1])])
                        j["ref"] = self._angle(j["ref"])
                        j["springref"] = self._angle(j["springref"])
                    if jt == JNT_FREE:
                        limited = False
                    n = np.linalg.norm(j["axis"])
                    j["axis"] = j["axis"] / n if n > MINVAL else np.array([0, 0, 1.0])
                    j["range"], j["limited"] = rng, limited
                    j["id"] = len(joints)
                    joints.append(j)
                    b["joints"].append(j["id"])
                elif ch.tag == "geom":
                    ga = self._attrs(ch, childcls, "geom")
                    gt = GEOM_TYPES[ga.get("type", "sphere")]
                    size = _floats(ga.get("size"), 3, [0, 0, 0])
                    pos = _floats(ga.get("pos"), 3, [0, 0, 0])
                    quat = self._orient(ga)
                    if "fromto" in ga and gt in (GEOM_CAPSULE, GEOM_CYLINDER, GEOM_BOX, GEOM_ELLIPSOID):
                        ft = _floats(ga["fromto"], 6)
                        p0, p1 = ft[:3], ft[3:]
                        pos = 0.5 * (p0 + p1)
                        quat = quat_z2vec(p1 - p0)
                        hl = 0.5 * float(np.linalg.norm(p1 - p0))
                        if gt in (GEOM_CAPSULE, GEOM_CYLINDER):
                            size[1] = hl
                        else:
                            size[2] = hl
                    g = dict(name=ga.get("name", ""), type=gt, body=bid, size=size, pos=pos, quat=quat,
                             contype=int(ga.get("contype", 1)), conaffinity=int(ga.get("conaffinity", 1)),
                             condim=int(ga.get("condim", 3)), priority=int(ga.get("priority", 0)),
                             friction=_floats(ga.get("friction"), 3, [1, 0.005, 0.0001]),
                             margin=float(ga.get("margin", 0)), gap=float(ga.get("gap", 0)),
                             solmix=float(ga.get("solmix", 1.0)),
                             solref=_floats(ga.get("solref"), 2, [0.02, 1.0]),
                             solimp=_floats(ga.get("solimp"), 5, [0.9, 0.95, 0.001, 0.5, 2.0]),
                             density=float(ga.get("density", 1000.0)),
                             mass=float(ga["mass"]) if "mass" in ga else None,
                             group=int(ga.get("group", 0)))
                    fr = _floats(ga.get("friction"), None, [1, 0.005, 0.0001])
                    if fr.size < 3:   # partial friction spec keeps the remaining defaults
                        fr = np.concatenate([fr, np.array([1, 0.005, 0.0001])[fr.size:]])
                    g["friction"] = fr[:3]
                    g["id"] = len(geoms)
                    geoms.append(g)
                    b["geoms"].append(g["id"])
                elif ch.tag == "site":
                    sa = self._attrs(ch, childcls, "site")
                    sites.append(dict(name=sa.get("name", ""), body=bid,
                                      pos=_floats(sa.get("pos"), 3, [0, 0, 0]), quat=self._orient(sa)))
                elif ch.tag == "inertial":
                    ia = dict(ch.attrib)
                    inr = dict(pos=_floats(ia.get("pos"), 3, [0, 0, 0]), quat=self._orient(ia),
                               mass=float(ia.get("mass", 0)))
                    if "diaginertia" in ia:
                        inr["inertia"] = _floats(ia["diaginertia"], 3)
                    elif "fullinertia" in ia:
                        f = _floats(ia["fullinertia"], 6)
                        I = np.array([[f[0], f[3], f[4]], [f[3], f[1], f[5]], [f[4], f[5], f[2]]])
                        w, V = np.linalg.eigh(I)
                        if np.linalg.det(V) < 0:
                            V[:, 2] = -V[:, 2]
                        inr["inertia"] = w
                        inr["quat"] = quat_mul(inr["quat"], mat2quat(V))
                    else:
                        inr["inertia"] = np.zeros(3)
                    b["inertial"] = inr
            # children bodies after this body's own elements: preorder DFS numbering
            for ch in elem:
                if ch.tag == "body":
                    walk(ch, bid, childcls)

        # geoms must be numbered body by body: we renumber after the walk
        wb = self.root.find("worldbody")
        walk(wb, -1, "main")
        order = []
        for b in bodies:
            order.extend(b["geoms"])
        remap = {old: new for new, old in enumerate(order)}
        geoms = [geoms[i] for i in order]
        for g in geoms:
            g["id"] = remap[g["id"]]
        for b in bodies:
            b["geoms"] = [remap[i] for i in b["geoms"]]

        # ---- joints / dofs in body order (joint ids are assigned in XML order = body order)
        nb = len(bodies)
        m.nbody, m.njnt, m.ngeom = nb, len(joints), len(geoms)
        qposadr, dofadr = [], []
        nq = nv = 0
        for j in joints:
            qposadr.append(nq)
            dofadr.append(nv)
            nq += {JNT_FREE: 7, JNT_BALL: 4}.get(j["type"], 1)
            nv += {JNT_FREE: 6, JNT_BALL: 3}.get(j["type"], 1)
        m.nq, m.nv = nq, nv

        body_parentid = np.array([b["parent"] for b in bodies], dtype=np.int32)
        body_parentid[0] = 0
        body_jntnum = np.array([len(b["joints"]) for b in bodies], dtype=np.int32)
        body_jntadr = np.array([b["joints"][0] if b["joints"] else -1 for b in bodies], dtype=np.int32)
        body_dofnum = np.zeros(nb, np.int32)
        body_dofadr = -np.ones(nb, np.int32)
        for i, b in enumerate(bodies):
            if b["joints"]:
                body_dofadr[i] = dofadr[b["joints"][0]]
                body_dofnum[i] = sum({JNT_FREE: 6, JNT_BALL: 3}.get(joints[j]["type"], 1) for j in b["joints"])
        body_geomnum = np.array([len(b["geoms"]) for b in bodies], dtype=np.int32)
        body_geomadr = np.array([b["geoms"][0] if b["geoms"] else -1 for b in bodies], dtype=np.int32)
        body_weldid = np.zeros(nb, np.int32)
        body_rootid = np.zeros(nb, np.int32)
        for i in range(1, nb):
            p = body_parentid[i]
            body_weldid[i] = i if body_jntnum[i] > 0 else body_weldid[p]
            body_rootid[i] = i if p == 0 else body_rootid[p]
        # subtree ranges in DFS order: subtree of i = [i, body_subtree_end[i])
        body_subtree_end = np.arange(1, nb + 1, dtype=np.int32)
        for i in range(nb - 1, 0, -1):
            p = body_parentid[i]
            body_subtree_end[p] = max(body_subtree_end[p], body_subtree_end[i])
        body_subtree_end[0] = nb
        body_depth = np.zeros(nb, np.int32)
        for i in range(1, nb):
            body_depth[i] = body_depth[body_parentid[i]] + 1

        # dof tables
        dof_bodyid = np.zeros(nv, np.int32)
        dof_jntid = np.zeros(nv, np.int32)
        dof_parentid = -np.ones(nv, np.int32)
        dof_armature = np.zeros(nv)
        dof_damping = np.zeros(nv)
        dof_frictionloss = np.zeros(nv)
        for jid, j in enumerate(joints):
            nd = {JNT_FREE: 6, JNT_BALL: 3}.get(j["type"], 1)
            for k in range(nd):
                d = dofadr[jid] + k
                dof_bodyid[d] = j["body"]
                dof_jntid[d] = jid
                dof_armature[d] = j["armature"]
                dof_damping[d] = j["damping"]
                dof_frictionloss[d] = j["frictionloss"]
        for d in range(nv):
            b = dof_bodyid[d]
            if d > 0 and dof_bodyid[d - 1] == b:
                dof_parentid[d] = d - 1
            else:
                p = body_parentid[b]
                while p > 0 and body_dofnum[p] == 0:
                    p = body_parentid[p]
                dof_parentid[d] = body_dofadr[p] + body_dofnum[p] - 1 if p > 0 else -1
        # sparse M layout (dof_Madr): row i = [M(i,i), M(i,parent), M(i,grandparent), ...]
        dof_Madr = np.zeros(nv, np.int32)
        dof_chainlen = np.zeros(nv, np.int32)
        adr = 0
        for i in range(nv):
            dof_Madr[i] = adr
            n, j = 0, i
            while j >= 0:
                n += 1
                j = dof_parentid[j]
            dof_chainlen[i] = n
            adr += n
        m.nM = adr
        # dof mask per body: bit d of word d//32 set if dof d is in the chain of body b
        nwords = max(1, (nv + 31) // 32)
        body_dofmask = np.zeros((nb, nwords), np.uint32)
        for b in range(1, nb):
            p = b
            while p > 0:
                for d in range(body_dofnum[p]):
                    dd = int(body_dofadr[p] + d)
                    body_dofmask[b, dd // 32] |= np.uint32(1 << (dd % 32))
                p = body_parentid[p]

        # joints arrays
        jnt_type = np.array([j["type"] for j in joints], np.int32)
        jnt_bodyid = np.array([j["body"] for j in joints], np.int32)
        jnt_qposadr = np.array(qposadr, np.int32)
        jnt_dofadr = np.array(dofadr, np.int32)
        jnt_limited = np.array([1 if j["limited"] else 0 for j in joints], np.int32)
        jnt_pos = np.array([j["pos"] for j in joints]).reshape(-1, 3)
        jnt_axis = np.array([j["axis"] for j in joints]).reshape(-1, 3)
        jnt_range = np.array([j["range"] for j in joints]).reshape(-1, 2)
        jnt_stiffness = np.array([j["stiffness"] for j in joints])
        jnt_margin = np.array([j["margin"] for j in joints])
        jnt_solref = np.array([j["solref"] for j in joints]).reshape(-1, 2)
        jnt_solimp = np.array([j["solimp"] for j in joints]).reshape(-1, 5)

        # qpos0 / qpos_spring
        qpos0 = np.zeros(nq)
        qpos_spring = np.zeros(nq)
        for jid, j in enumerate(joints):
            a = qposadr[jid]
            if j["type"] == JNT_FREE:
                b = bodies[j["body"]]
                qpos0[a:a + 3] = b["pos"]
                qpos0[a + 3:a + 7] = b["quat"]
                qpos_spring[a:a + 7] = qpos0[a:a + 7]
            elif j["type"] == JNT_BALL:
                qpos0[a:a + 4] = [1, 0, 0, 0]
                qpos_spring[a:a + 4] = [1, 0, 0, 0]
            else:
                qpos0[a] = j["ref"]
                qpos_spring[a] = j["springref"]
        # free-joint bodies: the body frame itself is carried by qpos (pos/quat reset to identity)
        body_pos = np.array([b["pos"] for b in bodies]).reshape(-1, 3)
        body_quat = np.array([b["quat"] for b in bodies]).reshape(-1, 4)

        # geoms arrays
        ng = len(geoms)
        geom_type = np.array([g["type"] for g in geoms], np.int32)
        geom_bodyid = np.array([g["body"] for g in geoms], np.int32)
        geom_contype = np.array([g["contype"] for g in geoms], np.int32)
        geom_conaffinity = np.array([g["conaffinity"] for g in geoms], np.int32)
        geom_condim = np.array([g["condim"] for g in geoms], np.int32)
        geom_priority = np.array([g["priority"] for g in geoms], np.int32)
        geom_size = np.array([g["size"][:3] for g in geoms]).reshape(-1, 3)
        geom_pos = np.array([g["pos"] for g in geoms]).reshape(-1, 3)
        geom_quat = np.array([g["quat"] for g in geoms]).reshape(-1, 4)
        geom_friction = np.array([g["friction"] for g in geoms]).reshape(-1, 3)
        geom_margin = np.array([g["margin"] for g in geoms])
        geom_gap = np.array([g["gap"] for g in geoms])
        geom_solmix = np.array([g["solmix"] for g in geoms])
        geom_solref = np.array([g["solref"] for g in geoms]).reshape(-1, 2)
        geom_solimp = np.array([g["solimp"] for g in geoms]).reshape(-1, 5)
        geom_rbound = np.array([_rbound(g["type"], g["size"]) for g in geoms])

        # ---- body inertia (inertiafromgeom)
        body_mass = np.zeros(nb)
        body_inertia = np.zeros((nb, 3))
        body_ipos = np.zeros((nb, 3))
        body_iquat = np.tile(np.array([1.0, 0, 0, 0]), (nb, 1))
        for i, b in enumerate(bodies):
            if i == 0:
                continue
            use_geoms = self.inertiafromgeom == "true" or (self.inertiafromgeom == "auto" and b["inertial"] is None)
            if b["inertial"] is not None and not (self.inertiafromgeom == "true"):
                inr = b["inertial"]
                body_mass[i] = inr["mass"]
                body_inertia[i] = inr["inertia"]
                body_ipos[i] = inr["pos"]
                body_iquat[i] = inr["quat"]
                continue
            if not use_geoms:
                continue
            parts = []
            for gid in b["geoms"]:
                g = geoms[gid]
                if g["type"] in (GEOM_PLANE, GEOM_HFIELD):
                    continue
                mvol, Iv = _geom_mass_inertia(g["type"], g["size"], 1.0)
                if g["mass"] is not None:
                    mass = g["mass"]
                    I = Iv * (mass / mvol) if mvol > 0 else np.zeros(3)
                else:
                    mass = g["density"] * mvol
                    I = Iv * g["density"]
                parts.append((mass, I, g["pos"], g["quat"]))
            if not parts:
                continue
            if len(parts) == 1:
                mass, I, p, q = parts[0]
                body_mass[i], body_inertia[i], body_ipos[i], body_iquat[i] = mass, I, p, q
                continue
            M = sum(pp[0] for pp in parts)
            com = sum(pp[0] * pp[2] for pp in parts) / max(M, MINVAL)
            Itot = np.zeros((3, 3))
            for mass, I, p, q in parts:
                R = quat2mat(q)
                Ig = R @ np.diag(I) @ R.T
                d = p - com
                Itot += Ig + mass * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
            w, V = np.linalg.eigh(Itot)
            if np.linalg.det(V) < 0:
                V[:, 2] = -V[:, 2]
            body_mass[i], body_inertia[i], body_ipos[i], body_iquat[i] = M, w, com, mat2quat(V)

        # ---- actuators
        acts = []
        act_el = self.root.find("actuator")
        if act_el is not None:
            for a in act_el:
                if a.tag not in ("motor", "position", "velocity", "general"):
                    continue
                aa = self._attrs(a, "main", a.tag)
                jname = aa.get("joint")
                jid = next((k for k, j in enumerate(joints) if j["name"] == jname), -1)
                gear = _floats(aa.get("gear"), 6, [1, 0, 0, 0, 0, 0])
                cr = _floats(aa.get("ctrlrange"), 2, [0, 0])
                fr = _floats(aa.get("forcerange"), 2, [0, 0])
                cl = aa.get("ctrllimited", "auto")
                fl = aa.get("forcelimited", "auto")
                ctrllimited = cl == "true" or (cl == "auto" and self.autolimits and "ctrlrange" in aa)
                forcelimited = fl == "true" or (fl == "auto" and self.autolimits and "forcerange" in aa)
                gain = np.zeros(3)
                bias = np.zeros(3)
                if a.tag == "motor":
                    gain[0] = 1.0
                elif a.tag == "position":
                    kp = float(aa.get("kp", 1.0))
                    kv = float(aa.get("kv", 0.0))
                    gain[0], bias[1], bias[2] = kp, -kp, -kv
                elif a.tag == "velocity":
                    kv = float(aa.get("kv", 1.0))
                    gain[0], bias[2] = kv, -kv
                else:
                    gain = _floats(aa.get("gainprm"), 3, [1, 0, 0])[:3]
                    bias = _floats(aa.get("biasprm"), 3, [0, 0, 0])[:3]
                acts.append(dict(name=aa.get("name", ""), jnt=jid, gear=gear[0], ctrllimited=int(ctrllimited),
                                 ctrlrange=cr, forcelimited=int(forcelimited), forcerange=fr,
                                 gain=gain, bias=bias))
        m.nu = len(acts)

        # ---- collision candidate pairs in MuJoCo order
        pairs = self._pairs(geoms, bodies, body_weldid, body_parentid, geom_type)

        A = m.arrays
        A.update(dict(
            body_parentid=body_parentid, body_rootid=body_rootid, body_weldid=body_weldid,
            body_jntnum=body_jntnum, body_jntadr=body_jntadr, body_dofnum=body_dofnum,
            body_dofadr=body_dofadr, body_geomnum=body_geomnum, body_geomadr=body_geomadr,
            body_subtree_end=body_subtree_end, body_depth=body_depth, body_dofmask=body_dofmask,
            body_pos=body_pos, body_quat=body_quat, body_ipos=body_ipos, body_iquat=body_iquat,
            body_mass=body_mass, body_inertia=body_inertia,
            jnt_type=jnt_type, jnt_bodyid=jnt_bodyid, jnt_qposadr=jnt_qposadr, jnt_dofadr=jnt_dofadr,
            jnt_limited=jnt_limited, jnt_pos=jnt_pos, jnt_axis=jnt_axis, jnt_range=jnt_range,
            jnt_stiffness=jnt_stiffness, jnt_margin=jnt_margin, jnt_solref=jnt_solref,
            jnt_solimp=jnt_solimp,
            dof_bodyid=dof_bodyid, dof_jntid=dof_jntid, dof_parentid=dof_parentid,
            dof_Madr=dof_Madr, dof_chainlen=dof_chainlen, dof_armature=dof_armature,
            dof_damping=dof_damping, dof_frictionloss=dof_frictionloss,
            geom_type=geom_type, geom_bodyid=geom_bodyid, geom_contype=geom_contype,
            geom_conaffinity=geom_conaffinity, geom_condim=geom_condim, geom_priority=geom_priority,
            geom_size=geom_size, geom_pos=geom_pos, geom_quat=geom_quat, geom_friction=geom_friction,
            geom_margin=geom_margin, geom_gap=geom_gap, geom_solmix=geom_solmix,
            geom_solref=geom_solref, geom_solimp=geom_solimp, geom_rbound=geom_rbound,
            qpos0=qpos0, qpos_spring=qpos_spring,
            actuator_trnid=np.array([a["jnt"] for a in acts], np.int32),
            actuator_gear=np.array([a["gear"] for a in acts]),
            actuator_ctrllimited=np.array([a["ctrllimited"] for a in acts], np.int32),
            actuator_ctrlrange=np.array([a["ctrlrange"] for a in acts]).reshape(-1, 2),
            actuator_forcelimited=np.array([a["forcelimited"] for a in acts], np.int32),
            actuator_forcerange=np.array([a["forcerange"] for a in acts]).reshape(-1, 2),
            actuator_gainprm=np.array([a["gain"] for a in acts]).reshape(-1, 3),
            actuator_biasprm=np.array([a["bias"] for a in acts]).reshape(-1, 3),
            site_bodyid=np.array([s["body"] for s in sites], np.int32),
            site_pos=np.array([s["pos"] for s in sites]).reshape(-1, 3),
            site_quat=np.array([s["quat"] for s in sites]).reshape(-1, 4),
        ))
        A.update(pairs)
        m.body_names = [b["name"] for b in bodies]
        m.jnt_names = [j["name"] for j in joints]
        m.geom_names = [g["name"] for g in geoms]
        m.actuator_names = [a["name"] for a in acts]
        m.site_names = [s["name"] for s in sites]
        _set_const(m)
        return m

    def _pairs(self, geoms, bodies, weldid, parentid, gtype):
        """Candidate contact pairs in MuJoCo's order: explicit <pair>s, then body pairs
        (b1 < b2) sorted by signature (b1<<16)+b2, geoms in body order (mj_collision
        [ext]). Parameters are mixed here once (condim/friction max, margin/gap max,
        solref/solimp by solmix), so the kernels read one record per pair."""
        out = []
        names = {g["name"]: g["id"] for g in geoms if g["name"]}
        excl = set()
        cont = self.root.find("contact")
        explicit = []
        if cont is not None:
            for c in cont:
                if c.tag == "exclude":
                    b1 = next(i for i, b in enumerate(bodies) if b["name"] == c.get("body1"))
                    b2 = next(i for i, b in enumerate(bodies) if b["name"] == c.get("body2"))
                    excl.add((min(b1, b2), max(b1, b2)))
                elif c.tag == "pair":
                    pa = self._attrs(c, "main", "pair")
                    g1, g2 = names[pa["geom1"]], names[pa["geom2"]]
                    rec = self._mix(geoms[g1], geoms[g2])
                    if "condim" in pa:
                        rec["condim"] = int(pa["condim"])
                    if "friction" in pa:
                        f = _floats(pa["friction"], 5)
                        rec["friction"] = f
                    if "margin" in pa:
                        rec["margin"] = float(pa["margin"])
                    if "gap" in pa:
                        rec["gap"] = float(pa["gap"])
                    if "solref" in pa:
                        rec["solref"] = _floats(pa["solref"], 2)
                    if "solimp" in pa:
                        rec["solimp"] = _floats(pa["solimp"], 5)
                    explicit.append((g1, g2, rec))
        for g1, g2, rec in explicit:
            out.append((g1, g2, rec, 1))
        nb = len(bodies)
        for b1 in range(nb):
            for b2 in range(b1 + 1, nb):
                w1, w2 = weldid[b1], weldid[b2]
                if w1 == w2:
                    continue
                wp1, wp2 = weldid[parentid[w1]], weldid[parentid[w2]]
                if w1 != 0 and w2 != 0 and (w1 == wp2 or w2 == wp1):
                    continue
                if (b1, b2) in excl:
                    continue
                for g1 in bodies[b1]["geoms"]:
                    for g2 in bodies[b2]["geoms"]:
                        ga, gb = geoms[g1], geoms[g2]
                        if not ((ga["contype"] & gb["conaffinity"]) or (gb["contype"] & ga["conaffinity"])):
                            continue
                        if gtype[g1] in (GEOM_PLANE,) and gtype[g2] in (GEOM_PLANE,):
                            continue
                        out.append((g1, g2, self._mix(ga, gb), 0))
        n = len(out)
        pair_geom = np.zeros((n, 2), np.int32)
        pair_condim = np.zeros(n, np.int32)
        pair_friction = np.zeros((n, 5))
        pair_margin = np.zeros(n)
        pair_gap = np.zeros(n)
        pair_solref = np.zeros((n, 2))
        pair_solimp = np.zeros((n, 5))
        pair_explicit = np.zeros(n, np.int32)
        for k, (g1, g2, rec, ex) in enumerate(out):
            # narrowphase convention: type(geom1) <= type(geom2) (mj_collideGeomPair swaps)
            if gtype[g1] > gtype[g2]:
                g1, g2 = g2, g1
            pair_geom[k] = (g1, g2)
            pair_condim[k] = rec["condim"]
            pair_friction[k] = rec["friction"]
            pair_margin[k] = rec["margin"]
            pair_gap[k] = rec["gap"]
            pair_solref[k] = rec["solref"]
            pair_solimp[k] = rec["solimp"]
            pair_explicit[k] = ex
        return dict(pair_geom=pair_geom, pair_condim=pair_condim, pair_friction=pair_friction,
                    pair_margin=pair_margin, pair_gap=pair_gap, pair_solref=pair_solref,
                    pair_solimp=pair_solimp, pair_explicit=pair_explicit)

    @staticmethod
    def _mix(ga, gb):
        if ga["priority"] != gb["priority"]:
            hi = ga if ga["priority"] > gb["priority"] else gb
            f = hi["friction"]
            return dict(condim=hi["condim"], friction=np.array([f[0], f[0], f[1], f[2], f[2]]),
                        margin=max(ga["margin"], gb["margin"]), gap=max(ga["gap"], gb["gap"]),
                        solref=hi["solref"].copy(), solimp=hi["solimp"].copy())
        f = np.maximum(ga["friction"], gb["friction"])
        s1, s2 = ga["solmix"], gb["solmix"]
        if s1 >= MINVAL and s2 >= MINVAL:
            mix = s1 / (s1 + s2)
        elif s1 < MINVAL and s2 < MINVAL:
            mix = 0.5
        else:
            mix = 1.0 if s1 >= MINVAL else 0.0
        if ga["solref"][0] > 0 and gb["solref"][0] > 0:
            solref = mix * ga["solref"] + (1 - mix) * gb["solref"]
        else:
            solref = np.minimum(ga["solref"], gb["solref"])
        solimp = mix * ga["solimp"] + (1 - mix) * gb["solimp"]
        return dict(condim=max(ga["condim"], gb["condim"]),
                    friction=np.array([f[0], f[0], f[1], f[2], f[2]]),
                    margin=max(ga["margin"], gb["margin"]), gap=max(ga["gap"], gb["gap"]),
                    solref=solref, solimp=solimp)


# ---------------------------------------------------------------------------------------
# mj_setConst at qpos0 (host fp64): kinematics + comPos + CRB, then invweight0/meaninertia
# ---------------------------------------------------------------------------------------
def _set_const(m: Model) -> None:
    A = m.arrays
    nb, nv = m.nbody, m.nv
    qpos = A["qpos0"].copy()
    xpos = np.zeros((nb, 3))
    xquat = np.tile([1.0, 0, 0, 0], (nb, 1))
    xmat = np.tile(np.eye(3), (nb, 1, 1))
    xanchor = np.zeros((m.njnt, 3))
    xaxis = np.zeros((m.njnt, 3))
    for i in range(1, nb):
        ja, jn = A["body_jntadr"][i], A["body_jntnum"][i]
        if jn == 1 and A["jnt_type"][ja] == JNT_FREE:
            a = A["jnt_qposadr"][ja]
            p = qpos[a:a + 3].copy()
            q = quat_normalize(qpos[a + 3:a + 7])
            xanchor[ja] = p
            xaxis[ja] = A["jnt_axis"][ja]
        else:
            par = A["body_parentid"][i]
            p = xmat[par] @ A["body_pos"][i] + xpos[par]
            q = quat_mul(xquat[par], A["body_quat"][i])
            for j in range(ja, ja + jn):
                a = A["jnt_qposadr"][j]
                R = quat2mat(q)
                xaxis[j] = R @ A["jnt_axis"][j]
                xanchor[j] = R @ A["jnt_pos"][j] + p
                t = A["jnt_type"][j]
                if t == JNT_SLIDE:
                    p = p + xaxis[j] * (qpos[a] - A["qpos0"][a])
                elif t in (JNT_HINGE, JNT_BALL):
                    ql = quat_normalize(qpos[a:a + 4]) if t == JNT_BALL else \
                        axis_angle_quat(A["jnt_axis"][j], qpos[a] - A["qpos0"][a])
                    q = quat_mul(q, ql)
                    p = xanchor[j] - quat2mat(q) @ A["jnt_pos"][j]
        q = quat_normalize(q)
        xpos[i], xquat[i], xmat[i] = p, q, quat2mat(q)
    xipos = np.array([xmat[i] @ A["body_ipos"][i] + xpos[i] for i in range(nb)])
    ximat = np.array([xmat[i] @ quat2mat(A["body_iquat"][i]) for i in range(nb)])
    mass = A["body_mass"]
    # subtree com
    sc = np.zeros((nb, 3))
    ms = np.zeros(nb)
    for i in range(nb - 1, -1, -1):
        sc[i] += xipos[i] * mass[i]
        ms[i] += mass[i]
        if i:
            sc[A["body_parentid"][i]] += sc[i]
            ms[A["body_parentid"][i]] += ms[i]
        sc[i] = xipos[i] if ms[i] < MINVAL else sc[i] / max(MINVAL, ms[i])
    # 6D cdof (rot; lin) about subtree com of the root
    cdof = np.zeros((nv, 6))
    for d in range(nv):
        b = A["dof_bodyid"][d]
        j = A["dof_jntid"][d]
        t = A["jnt_type"][j]
        off = sc[A["body_rootid"][b]] - xanchor[j]
        k = d - A["jnt_dofadr"][j]
        if t == JNT_FREE and k < 3:
            cdof[d, 3 + k] = 1.0
        elif t in (JNT_FREE, JNT_BALL):
            kk = k - 3 if t == JNT_FREE else k
            ax = xmat[b][:, kk]
            cdof[d, :3] = ax
            cdof[d, 3:] = np.cross(ax, off)
        elif t == JNT_SLIDE:
            cdof[d, 3:] = xaxis[j]
        else:
            cdof[d, :3] = xaxis[j]
            cdof[d, 3:] = np.cross(xaxis[j], off)
    # spatial inertia about subtree com (6x6 blocks), composite
    def sp_inertia(i):
        R = ximat[i]
        I = R @ np.diag(A["body_inertia"][i]) @ R.T
        dvec = xipos[i] - sc[A["body_rootid"][i]]
        mI = mass[i]
        cx = np.array([[0, -dvec[2], dvec[1]], [dvec[2], 0, -dvec[0]], [-dvec[1], dvec[0], 0]])
        top = I - mI * cx @ cx
        return np.block([[top, mI * cx], [-mI * cx, mI * np.eye(3)]])
    crb = [np.zeros((6, 6))] + [sp_inertia(i) for i in range(1, nb)]
    for i in range(nb - 1, 0, -1):
        p = A["body_parentid"][i]
        if p > 0:
            crb[p] = crb[p] + crb[i]
    M = np.zeros((nv, nv))
    for i in range(nv):
        buf = crb[A["dof_bodyid"][i]] @ cdof[i]
        j = i
        while j >= 0:
            M[i, j] = M[j, i] = cdof[j] @ buf
            j = A["dof_parentid"][j]
        M[i, i] += A["dof_armature"][i]
    m.meaninertia = float(np.trace(M) / nv) if nv else 1.0
    Minv = np.linalg.inv(M) if nv else np.zeros((0, 0))
    # body_invweight0: mean diagonal of J M^-1 J' blocks at the body com
    biw = np.zeros((nb, 2))
    for i in range(1, nb):
        if A["body_weldid"][i] == 0:
            continue
        J = np.zeros((6, nv))
        off = xipos[i] - sc[A["body_rootid"][i]]
        for d in range(nv):
            if int(A["body_dofmask"][i, d // 32]) >> (d % 32) & 1:
                J[:3, d] = cdof[d, 3:] + np.cross(cdof[d, :3], off)
                J[3:, d] = cdof[d, :3]
        Am = J @ Minv @ J.T
        biw[i, 0] = max(MINVAL, (Am[0, 0] + Am[1, 1] + Am[2, 2]) / 3)
        biw[i, 1] = max(MINVAL, (Am[3, 3] + Am[4, 4] + Am[5, 5]) / 3)
    diw = np.zeros(nv)
    for j in range(m.njnt):
        a = A["jnt_dofadr"][j]
        t = A["jnt_type"][j]
        if t == JNT_FREE:
            diw[a:a + 3] = np.mean(np.diag(Minv)[a:a + 3])
            diw[a + 3:a + 6] = np.mean(np.diag(Minv)[a + 3:a + 6])
        elif t == JNT_BALL:
            diw[a:a + 3] = np.mean(np.diag(Minv)[a:a + 3])
        else:
            diw[a] = Minv[a, a]
    A["body_invweight0"] = biw
    A["dof_invweight0"] = diw


def compile_xml(xml: str, name: str = "") -> Model:
    """Compile an MJCF string (the reference builds one per env, e.g. soccer_env.py:220)."""
    return _Compiler(xml).compile(name)
