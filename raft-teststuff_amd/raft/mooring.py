"""Quasi-static mooring: the MoorPy-equivalent statics RAFT's solveStatics and outputs use
(SURVEY.md §8(f) row 2).

The reference delegates mooring to MoorPy (third-party, unpinned in the reference's
pyproject.toml:53-62, absent from this image).  Its call sites are:
  * FOWT.__init__ builds a System from design['mooring'] (raft/raft_fowt.py:166-189):
    parseYAML, one coupled Body carrying the 'vessel' points, transform(x_ref, y_ref,
    heading_adjust), initialize;
  * FOWT.setPosition moves the body and reads C_moor = getCoupledStiffnessA() and
    F_moor0 = body.getForces(lines_only=True) (raft/raft_fowt.py:275-288);
  * Model.solveStatics' Newton step uses getCoupledStiffnessA(lines_only=True)
    (raft/raft_model.py:686-700); analyzeUnloaded reads getCoupledStiffness(lines_only=True)
    and getForces (:204-214);
  * saveTurbineOutputs / analyzeCases read getCoupledStiffness(tensions=True) (the tension
    Jacobian J_moor) and getTensions() (raft/raft_fowt.py:1878-1898, raft/raft_model.py:346-388);
  * the array-level System of a farm is loaded from a MoorDyn-style file
    (raft/raft_model.py:83-100) and has free points solved by solveEquilibrium.

This module restates the published algorithm those calls rely on:
  * the elastic catenary of a line with optional seabed contact (Jonkman's quasi-static
    formulation, FAST v7 `Catenary`, which MoorPy adopts), Newton on (HF, VF);
  * the analytic end stiffness inv(d(XF, ZF)/d(HF, VF)) plus the transverse HF/XF term;
  * rigid-body assembly of point forces and stiffness onto the 6 coupled DOFs (with the
    geometric term of the attachment lever arms);
  * a Newton equilibrium of free points.
Parity is pinned only through the reference's own solveStatics / solveEigen expectations
(tests/test_model.py:62-204, reproduced by tests/test_mooring.py); beyond those values it is
unpinned.
"""
import math

import numpy as np

RHO = 1025.0
G = 9.81


def get_h(r):
    """Alternator matrix: get_h(r) @ v = v x r (raft/helpers.py:346-355)."""
    return np.array([[0.0, r[2], -r[1]], [-r[2], 0.0, r[0]], [r[1], -r[0], 0.0]])


def rotation_matrix(x3, x2, x1):
    """Intrinsic z-y-x rotation (roll x3, pitch x2, yaw x1), raft/helpers.py:357-384."""
    s1, c1 = math.sin(x1), math.cos(x1)
    s2, c2 = math.sin(x2), math.cos(x2)
    s3, c3 = math.sin(x3), math.cos(x3)
    return np.array([[c1 * c2, c1 * s2 * s3 - c3 * s1, s1 * s3 + c1 * c3 * s2],
                     [c2 * s1, c1 * c3 + s1 * s2 * s3, c3 * s1 * s2 - c1 * s3],
                     [-s2, c2 * s3, c2 * c3]])


# ------------------------------------------------------------------------------ catenary
def catenary(XF, ZF, L, EA, W, CB=0.0, Tol=1e-6, MaxIter=100, HF0=0.0, VF0=0.0):
    """Elastic catenary between anchor end A and end B (B is XF horizontally and ZF
    vertically from A).  Returns (HA, VA, HF, VF, K) with the horizontal/vertical tension
    components at A and B (B is pulled toward A with (HF, VF) downward) and
    K = d(HF, VF)/d(XF, ZF), the 2x2 end-B stiffness.
    CB < 0: no seabed contact possible; CB >= 0: seabed friction coefficient.
    Newton on (HF, VF) from the previous solution when given (warm start) or the Peyrot &
    Goulois guess; the iteration stops BEFORE applying a step below Tol (relative), as the
    FAST v7 routine MoorPy follows does.  That detail sets the returned tensions at the
    ~Tol level, and the reference's solveStatics offsets depend on it at the 1e-5 level
    (tests/test_mooring.py reproduces them to ~1e-9 with it, to ~1e-5 without)."""
    if W < 0:
        raise NotImplementedError("buoyant mooring lines")
    if XF < 0 or L <= 0 or EA <= 0:
        raise ValueError(f"catenary: XF={XF}, L={L}, EA={EA}")
    WL = W * L
    WEA = W * EA
    LOvrEA = L / EA
    CBOvrEA = CB / EA
    if HF0 > 0 and VF0 > 0:
        HF, VF = HF0, VF0
    else:                                   # Peyrot & Goulois initial guess (as FAST v7)
        if XF == 0.0:
            lam = 1.0e6
        elif L <= math.sqrt(XF * XF + ZF * ZF):
            lam = 0.2
        else:
            lam = math.sqrt(3.0 * ((L * L - ZF * ZF) / (XF * XF) - 1.0))
        HF = max(abs(0.5 * W * XF / lam), Tol)
        VF = 0.5 * W * (ZF / math.tanh(lam) + L)
    for _ in range(MaxIter):
        EXF, EZF, J = _catenary_residual(XF, ZF, L, EA, W, CB, HF, VF, WL, WEA, LOvrEA, CBOvrEA)
        det = J[0][0] * J[1][1] - J[0][1] * J[1][0]
        dHF = (-J[1][1] * EXF + J[0][1] * EZF) / det
        dVF = (J[1][0] * EXF - J[0][0] * EZF) / det
        dHF = max(dHF, (Tol - 1.0) * HF)          # keep HF positive
        if abs(dHF) <= abs(Tol * HF) and abs(dVF) <= abs(Tol * VF):
            break                                  # converged: the last (small) step is not applied
        HF += dHF
        VF += dVF
    else:
        if HF0 > 0 and VF0 > 0:           # a warm start far from this shape: retry from the
            return catenary(XF, ZF, L, EA, W, CB, Tol, MaxIter)   # default guess, as MoorPy does
        raise RuntimeError(f"catenary did not converge (XF={XF}, ZF={ZF}, L={L})")
    K = np.array([[J[1][1], -J[0][1]], [-J[1][0], J[0][0]]]) / det     # inv(J)
    VFMWL = VF - WL
    if CB < 0 or VFMWL > 0:
        HA, VA = HF, VFMWL
    elif -CB * VFMWL < HF:
        HA, VA = HF + CB * VFMWL, 0.0
    else:
        HA, VA = 0.0, 0.0
    return HA, VA, HF, VF, K


def _catenary_residual(XF, ZF, L, EA, W, CB, HF, VF, WL, WEA, LOvrEA, CBOvrEA):
    """(EXF, EZF, J = d(XF, ZF)/d(HF, VF)) of Jonkman's catenary equations."""
    VFMWL = VF - WL
    HF_W = HF / W
    VF_HF = VF / HF
    VFMWL_HF = VFMWL / HF
    VF_HF2 = VF_HF * VF_HF
    VFMWL_HF2 = VFMWL_HF * VFMWL_HF
    S1 = math.sqrt(1.0 + VF_HF2)
    S2 = math.sqrt(1.0 + VFMWL_HF2)
    if CB < 0.0 or VFMWL > 0.0:                               # fully suspended
        lg = math.log(VF_HF + S1) - math.log(VFMWL_HF + S2)
        EXF = lg * HF_W + LOvrEA * HF - XF
        EZF = (S1 - S2) * HF_W + LOvrEA * (VF - 0.5 * WL) - ZF
        dXFdHF = lg / W - ((VF_HF + VF_HF2 / S1) / (VF_HF + S1) - (VFMWL_HF + VFMWL_HF2 / S2) / (VFMWL_HF + S2)) / W \
            + LOvrEA
        dXFdVF = ((1.0 + VF_HF / S1) / (VF_HF + S1) - (1.0 + VFMWL_HF / S2) / (VFMWL_HF + S2)) / W
        dZFdHF = (S1 - S2) / W - (VF_HF2 / S1 - VFMWL_HF2 / S2) / W
        dZFdVF = (VF_HF / S1 - VFMWL_HF / S2) / W + LOvrEA
    elif -CB * VFMWL < HF:                                    # on the seabed, anchor tension > 0
        LB = L - VF / W
        lg = math.log(VF_HF + S1)
        EXF = lg * HF_W - 0.5 * CBOvrEA * W * LB * LB + LOvrEA * HF + LB - XF
        EZF = (S1 - 1.0) * HF_W + 0.5 * VF * VF / WEA - ZF
        dXFdHF = lg / W - ((VF_HF + VF_HF2 / S1) / (VF_HF + S1)) / W + LOvrEA
        dXFdVF = ((1.0 + VF_HF / S1) / (VF_HF + S1)) / W + CBOvrEA * LB - 1.0 / W
        dZFdHF = (S1 - 1.0 - VF_HF2 / S1) / W
        dZFdVF = (VF_HF / S1) / W + VF / WEA
    else:                                                     # on the seabed, anchor tension 0
        LB = L - VF / W
        lg = math.log(VF_HF + S1)
        x = LB - HF_W / CB
        EXF = lg * HF_W - 0.5 * CBOvrEA * W * (LB * LB - x * x) + LOvrEA * HF + LB - XF
        EZF = (S1 - 1.0) * HF_W + 0.5 * VF * VF / WEA - ZF
        dXFdHF = lg / W - ((VF_HF + VF_HF2 / S1) / (VF_HF + S1)) / W + LOvrEA - x / EA
        dXFdVF = ((1.0 + VF_HF / S1) / (VF_HF + S1)) / W + HF / WEA - 1.0 / W
        dZFdHF = (S1 - 1.0 - VF_HF2 / S1) / W
        dZFdVF = (VF_HF / S1) / W + VF / WEA
    return EXF, EZF, ((dXFdHF, dXFdVF), (dZFdHF, dZFdVF))


# ------------------------------------------------------------------------------ objects
class Point:
    FIXED, COUPLED, FREE = 1, -1, 0

    def __init__(self, number, ptype, r, m=0.0, v=0.0):
        self.number = number
        self.type = ptype
        self.r = np.array(r, dtype=float)
        self.m, self.v = float(m), float(v)
        self.lines = []          # (line, end) with end 'A' or 'B'


class Line:
    def __init__(self, number, L, ltype, pA, pB):
        self.number = number
        self.L = float(L)
        self.type = ltype
        self.pA, self.pB = pA, pB
        self.HF = self.VF = 0.0          # warm start of the next catenary solve
        self.fA = np.zeros(3)            # force of the line on its end points
        self.fB = np.zeros(3)
        self.KA = self.KB = self.KAB = np.zeros([3, 3])
        self.TA = self.TB = 0.0

    def current_load(self, U, rho=RHO):
        """Mean drag of a uniform current U on the line, per unit (unstretched) length, on the
        straight chord between its ends: transverse 0.5 rho d Cd |Un| Un plus tangential
        0.5 rho pi d CdAx |Ut| Ut (the MoorDyn drag convention of the line-type table).
        MoorPy's currentMod = 1 (raft/raft_model.py:561-577) applies a current this way; its
        exact form is not visible from the reference, so this is parity unpinned."""
        U = np.asarray(U, dtype=float)
        if not np.any(U):
            return np.zeros(3)
        d = self.pB.r - self.pA.r
        n = np.linalg.norm(d)
        q = d / n if n > 0 else np.array([0.0, 0.0, 1.0])
        Ut = np.dot(U, q) * q
        Un = U - Ut
        dia = self.type["d"]
        return (0.5 * rho * dia * self.type.get("Cd", 0.0) * np.linalg.norm(Un) * Un
                + 0.5 * rho * math.pi * dia * self.type.get("CdAx", 0.0) * np.linalg.norm(Ut) * Ut)

    def static_solve(self, depth, tol=1e-6, current=None, rho=RHO):
        """End forces and 3-D end stiffness for the current end positions.  The catenary is
        solved from the lower end (anchor side) to the upper end; the forces on the ends are
        the line's pull: the upper end toward the lower one and down, the lower end toward
        the upper one (zero vertical force where the line rests on the seabed).
        With a uniform `current`, the distributed load is the wet weight plus the line's
        current drag (current_load); the catenary is solved in the frame whose -z axis is that
        load's direction, with the same seabed-contact rule (the seabed plane then taken
        normal to the load through the lower end), and forces and stiffness are rotated back.
        Zero current gives the plain solve bit for bit.
        Approximation (parity unpinned): with current, the ends of EVERY line are
        ordered by height along the load, not by global depth (the catenary hangs "below" the
        end that is upstream of the load), and seabed contact is decided from the global depth
        of the end that ordering calls lower, as without current.  So a heavy line whose load
        current tilts far enough toward the fairlead (the anchor then ranks upper) is solved
        fully suspended, whatever the anchor's depth; a net load that points away from the
        seabed (a buoyant line in current) never has seabed contact
        (tests/test_mooring.py::test_heavy_line_ordering_flip_in_current)."""
        W = self.type["w"]
        R = None
        up = False                                     # the net load points away from the seabed
        if current is not None and np.any(current):
            f = np.array([0.0, 0.0, -W]) + self.current_load(current, rho)
            W = float(np.linalg.norm(f))
            a = f / W                                  # load direction -> (0, 0, -1)
            up = a[2] > 0.0
            # a load with an upward component is first turned 180 deg about x, so that the
            # Rodrigues step is taken at 1 + cos >= 1 (it is singular for a load straight up)
            R0 = np.diag([1.0, -1.0, -1.0]) if up else np.eye(3)
            a = R0 @ a
            v = np.array([a[1] * -1.0 - a[2] * 0.0, a[2] * 0.0 - a[0] * -1.0, 0.0])   # a x (0, 0, -1)
            cth = -a[2]
            V = np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])
            R = (np.eye(3) + V + V @ V / (1.0 + cth)) @ R0   # R f / |f| = (0, 0, -1)
        zA, zB = (self.pA.r[2], self.pB.r[2]) if R is None else ((R @ self.pA.r)[2], (R @ self.pB.r)[2])
        swap = zB < zA
        lower, upper = (self.pB, self.pA) if swap else (self.pA, self.pB)
        d = upper.r - lower.r
        if R is not None:
            d = R @ d
        LH = math.hypot(d[0], d[1])
        c, s = (d[0] / LH, d[1] / LH) if LH > 0 else (0.0, 0.0)
        if up:
            CB = -1.0                                  # pulled away from the seabed: never in contact
        else:
            CB = -depth - lower.r[2] if lower.r[2] > -depth else 0.0    # off the seabed: no contact
        HA, VA, HF, VF, K2 = catenary(LH, d[2], self.L, self.type["EA"], W, CB=CB,
                                       HF0=self.HF, VF0=self.VF, Tol=tol)
        self.HF, self.VF = HF, VF
        f_up = np.array([-HF * c, -HF * s, -VF])
        f_lo = np.array([HA * c, HA * s, VA])
        Kt = HF / LH if LH > 0 else 0.0                          # transverse (geometric) stiffness
        Kxx, Kxz, Kzx, Kzz = K2[0, 0], K2[0, 1], K2[1, 0], K2[1, 1]
        Ku = np.array([[c * c * Kxx + s * s * Kt, c * s * (Kxx - Kt), c * Kxz],
                       [c * s * (Kxx - Kt), s * s * Kxx + c * c * Kt, s * Kxz],
                       [c * Kzx, s * Kzx, Kzz]])
        if R is not None:                                        # back to the global frame
            f_up, f_lo = R.T @ f_up, R.T @ f_lo
            Ku = R.T @ Ku @ R
        self.fA, self.fB = (f_up, f_lo) if swap else (f_lo, f_up)
        self.TA = float(np.linalg.norm(self.fA))
        self.TB = float(np.linalg.norm(self.fB))
        # the end forces depend on the end separation only (line weight and, for a fixed
        # anchor, the seabed reaction aside): both ends see Ku, the cross term is -Ku
        self.KA = Ku
        self.KB = Ku
        self.KAB = -Ku


class Body:
    def __init__(self, number, r6):
        self.number = number
        self.r6 = np.array(r6, dtype=float)
        self.points = []          # (Point, rRel)

    def attach(self, point, r_rel):
        self.points.append((point, np.array(r_rel, dtype=float)))

    def set_position(self, r6):
        self.r6 = np.array(r6, dtype=float)
        R = rotation_matrix(*self.r6[3:])
        for p, rr in self.points:
            p.r = self.r6[:3] + R @ rr


class MooringSystem:
    """A quasi-static mooring system: fixed, coupled (body-attached) and free points joined
    by catenary lines; one or more coupled bodies (one per FOWT)."""

    def __init__(self, depth=0.0, rho=RHO, g=G, cat_tol=1e-5):
        self.depth = float(depth)
        self.cat_tol = cat_tol            # relative tolerance of the catenary solves
        self.free_tol = 0.05              # free-point equilibrium step tolerance [m]
        self.rho, self.g = rho, g
        self.current = np.zeros(3)        # uniform current [m/s] on the lines (MoorPy currentMod 1)
        self.points, self.lines, self.bodies = [], [], []
        self.line_types = {}

    # ----------------------------------------------------------------- construction
    def add_line_type(self, name, d, m, EA, Cd=0.0, CdAx=0.0):
        w = (m - self.rho * math.pi / 4.0 * d * d) * self.g       # wet weight per length
        self.line_types[name] = dict(name=name, d=float(d), m=float(m), EA=float(EA), w=w, Cd=float(Cd),
                                     CdAx=float(CdAx))

    def add_point(self, ptype, r, m=0.0, v=0.0):
        p = Point(len(self.points) + 1, ptype, r, m, v)
        self.points.append(p)
        return p

    def add_line(self, L, ltype, pA, pB):
        ln = Line(len(self.lines) + 1, L, self.line_types[ltype], pA, pB)
        self.lines.append(ln)
        pA.lines.append((ln, "A"))
        pB.lines.append((ln, "B"))
        return ln

    def add_body(self, r6):
        b = Body(len(self.bodies) + 1, r6)
        self.bodies.append(b)
        return b

    @classmethod
    def from_yaml(cls, d):
        """A System from the design's `mooring` section (points / lines / line_types) with one
        coupled body at the origin carrying the 'vessel' points (raft/raft_fowt.py:166-186)."""
        ms = cls(depth=float(d["water_depth"]))
        for lt in d.get("line_types", []):
            ms.add_line_type(lt["name"], float(lt["diameter"]), float(lt["mass_density"]), float(lt["stiffness"]),
                             float(lt.get("transverse_drag", 0.0)), float(lt.get("tangential_drag", 0.0)))
        body = ms.add_body(np.zeros(6))
        names = {}
        for pd in d.get("points", []):
            t = str(pd.get("type", "fixed")).lower()
            ptype = {"fixed": Point.FIXED, "anchor": Point.FIXED, "vessel": Point.COUPLED, "coupled": Point.COUPLED,
                     "fairlead": Point.COUPLED, "free": Point.FREE, "connection": Point.FREE}.get(t)
            if ptype is None:
                raise ValueError(f"mooring point type '{t}' not recognised")
            p = ms.add_point(ptype, np.asarray(pd["location"], dtype=float), pd.get("mass", 0.0), pd.get("volume", 0.0))
            names[pd["name"]] = p
            if ptype == Point.COUPLED:
                body.attach(p, p.r.copy())
                p.type = Point.FIXED                 # fixed to the body (raft/raft_fowt.py:175-177)
        for ld in d.get("lines", []):
            ms.add_line(float(ld["length"]), ld["type"], names[ld["endA"]], names[ld["endB"]])
        return ms

    def load_moordyn(self, path):
        """Line types, points and lines of a MoorDyn-style input file (the array-level system
        of raft/raft_model.py:83-100).  'TurbineN' points attach to body N (added before),
        'Fixed' points are anchors, 'Free' points are solved for equilibrium."""
        section = None
        with open(path) as fh:
            lines = fh.read().splitlines()
        for raw in lines:
            s = raw.split("#")[0].strip()
            if not s:
                continue
            if s.startswith("---"):
                up = s.upper()
                section = ("types" if "LINE TYPES" in up else "points" if "POINTS" in up else
                           "lines" if "LINES" in up else "options" if "OPTIONS" in up else "other")
                continue
            tok = s.split()
            if section == "types" and len(tok) >= 4 and _isnum(tok[1]):   # Name Diam Mass/m EA BA EI Cd Ca CdAx CaAx
                self.add_line_type(tok[0], float(tok[1]), float(tok[2]), float(tok[3]),
                                   float(tok[6]) if len(tok) > 6 else 0.0, float(tok[8]) if len(tok) > 8 else 0.0)
            elif section == "points" and len(tok) >= 5 and _isnum(tok[0]):
                att = tok[1].lower()
                r = np.array([float(tok[2]), float(tok[3]), float(tok[4])])
                m = float(tok[5]) if len(tok) > 5 else 0.0
                v = float(tok[6]) if len(tok) > 6 else 0.0
                if att.startswith("turbine") or att.startswith("body"):
                    b = self.bodies[int("".join(ch for ch in att if ch.isdigit())) - 1]
                    p = self.add_point(Point.FIXED, b.r6[:3] + r, m, v)
                    b.attach(p, r)
                elif att in ("fixed", "anchor"):
                    self.add_point(Point.FIXED, r, m, v)
                else:
                    self.add_point(Point.FREE, r, m, v)
            elif section == "lines" and len(tok) >= 5 and _isnum(tok[0]):
                self.add_line(float(tok[4]), tok[1], self.points[int(tok[2]) - 1], self.points[int(tok[3]) - 1])
            elif section == "options" and len(tok) >= 2 and tok[1].lower() in ("wtrdpth", "depth"):
                self.depth = float(tok[0])

    def transform(self, trans=(0.0, 0.0), rot=0.0):
        """Rotate the whole system about z by `rot` degrees, then translate horizontally
        (FOWT placement, raft/raft_fowt.py:185)."""
        c, s = math.cos(math.radians(rot)), math.sin(math.radians(rot))
        R = np.array([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]])
        t = np.array([trans[0], trans[1], 0.0])
        for p in self.points:
            p.r = R @ p.r + t
        for b in self.bodies:
            b.points = [(p, R @ rr) for p, rr in b.points]
            b.r6 = b.r6.copy()
            b.r6[:3] = b.r6[:3] + t

    def initialize(self):
        for b in self.bodies:
            b.set_position(b.r6)
        self.solve_equilibrium()

    # ----------------------------------------------------------------- statics
    def _solve_lines(self):
        cur = self.current if np.any(self.current) else None
        for ln in self.lines:
            ln.static_solve(self.depth, self.cat_tol, cur, self.rho)

    def point_force(self, p, lines_only=False):
        f = np.zeros(3)
        for ln, end in p.lines:
            f += ln.fA if end == "A" else ln.fB
        if not lines_only:
            f[2] += -p.m * self.g + p.v * self.rho * self.g
        return f

    def point_stiffness(self, p):
        K = np.zeros([3, 3])
        for ln, end in p.lines:
            K += ln.KA if end == "A" else ln.KB
        return K

    def _free_stiffness(self, free, idx):
        n = 3 * len(free)
        K = np.zeros([n, n])
        for ln in self.lines:
            ia, ib = idx.get(ln.pA.number), idx.get(ln.pB.number)
            if ia is not None:
                K[3 * ia:3 * ia + 3, 3 * ia:3 * ia + 3] += ln.KA
            if ib is not None:
                K[3 * ib:3 * ib + 3, 3 * ib:3 * ib + 3] += ln.KB
            if ia is not None and ib is not None:
                K[3 * ia:3 * ia + 3, 3 * ib:3 * ib + 3] += ln.KAB
                K[3 * ib:3 * ib + 3, 3 * ia:3 * ia + 3] += ln.KAB.T
        return K

    def solve_equilibrium(self, tol=None, maxIter=500):
        """Lines at the current body positions; free points moved to force equilibrium
        (System.solveEquilibrium: dsolve2 on the free-point coordinates with Newton steps on
        the analytic line stiffness, each step limited to depth/10; converged when every
        step is below `tol`, default self.free_tol)."""
        from .dsolve import dsolve2
        free = [p for p in self.points if p.type == Point.FREE]
        self._solve_lines()
        if not free:
            return
        idx = {p.number: i for i, p in enumerate(free)}
        tol = self.free_tol if tol is None else tol

        def eval_func(X, args):
            for p in free:
                p.r = X[3 * idx[p.number]:3 * idx[p.number] + 3].copy()
            self._solve_lines()
            return np.concatenate([self.point_force(p) for p in free]), {}, False

        def step_func(X, args, Y, oths, Ytarget, err, tol_, it, maxIter_):
            dX = np.linalg.solve(self._free_stiffness(free, idx), Y)
            lim = self.depth / 10 if self.depth > 0 else 10.0
            big = np.abs(dX).max()
            return dX * (lim / big) if big > lim else dX

        X0 = np.concatenate([p.r for p in free])
        X, Y, info = dsolve2(eval_func, X0, step_func=step_func, tol=tol, maxIter=maxIter)
        eval_func(X, None)

    def set_body_positions(self, r6s):
        for b, r6 in zip(self.bodies, r6s):
            b.set_position(r6)
        self.solve_equilibrium()

    def body_forces(self, b, lines_only=True):
        """Net mooring force and moment on a body about its reference point (getForces)."""
        F = np.zeros(6)
        for p, rr in b.points:
            f = self.point_force(p, lines_only=lines_only)
            r = p.r - b.r6[:3]
            F[:3] += f
            F[3:] += np.cross(r, f)
        return F

    def coupled_forces(self, lines_only=True):
        return np.concatenate([self.body_forces(b, lines_only) for b in self.bodies])

    def coupled_stiffness_analytic(self):
        """6nb x 6nb stiffness of the coupled body DOFs, analytic (getCoupledStiffnessA):
        point stiffness carried by the lever arms plus the geometric term of the attachment
        forces; free points are condensed out."""
        nb = len(self.bodies)
        free = [p for p in self.points if p.type == Point.FREE]
        owner = {}
        for ib, b in enumerate(self.bodies):
            for p, _ in b.points:
                owner[p.number] = ib
        # T maps body DOFs to attached-point displacements (3 per point)
        att = [(p, ib, p.r - self.bodies[ib].r6[:3]) for ib, b in enumerate(self.bodies) for p, _ in b.points]
        na, nf = len(att), len(free)
        K = np.zeros([6 * nb, 6 * nb])
        for p, ib, r in att:                      # geometric (lever-arm rotation) term
            f = self.point_force(p, lines_only=True)
            K[6 * ib + 3:6 * ib + 6, 6 * ib + 3:6 * ib + 6] += -get_h(f) @ get_h(r)
        # point-level stiffness over attached + free points
        ids = [p.number for p, _, _ in att] + [p.number for p in free]
        pos = {pid: i for i, pid in enumerate(ids)}
        Kp = np.zeros([3 * len(ids), 3 * len(ids)])
        for ln in self.lines:
            ia, ib_ = pos.get(ln.pA.number), pos.get(ln.pB.number)
            if ia is not None:
                Kp[3 * ia:3 * ia + 3, 3 * ia:3 * ia + 3] += ln.KA
            if ib_ is not None:
                Kp[3 * ib_:3 * ib_ + 3, 3 * ib_:3 * ib_ + 3] += ln.KB
            if ia is not None and ib_ is not None:
                Kp[3 * ia:3 * ia + 3, 3 * ib_:3 * ib_ + 3] += ln.KAB
                Kp[3 * ib_:3 * ib_ + 3, 3 * ia:3 * ia + 3] += ln.KAB.T
        T = np.zeros([3 * na, 6 * nb])
        for i, (p, ib, r) in enumerate(att):
            T[3 * i:3 * i + 3, 6 * ib:6 * ib + 3] = np.eye(3)
            T[3 * i:3 * i + 3, 6 * ib + 3:6 * ib + 6] = get_h(r)     # displacement of theta x r
        Kaa = Kp[:3 * na, :3 * na]
        if nf:
            Kaf = Kp[:3 * na, 3 * na:]
            Kff = Kp[3 * na:, 3 * na:]
            Kaa = Kaa - Kaf @ np.linalg.solve(Kff, Kaf.T)
        K += T.T @ Kaa @ T
        return K

    def tensions(self):
        """Line end tensions [TA_1..TA_n, TB_1..TB_n] (getTensions)."""
        return np.array([ln.TA for ln in self.lines] + [ln.TB for ln in self.lines])

    def coupled_stiffness_fd(self, dx=0.1, dth=0.1, tensions=False):
        """Central-difference stiffness of the coupled DOFs (getCoupledStiffness, lines only)
        and optionally the tension Jacobian dT/dX [2 nLines, 6 nb]."""
        nb = len(self.bodies)
        X0 = [b.r6.copy() for b in self.bodies]
        saved = [p.r.copy() for p in self.points]
        warm = [(ln.HF, ln.VF) for ln in self.lines]

        def restore():             # every perturbed solve starts from the same state: deterministic
            for p, r in zip(self.points, saved):
                p.r = r.copy()
            for ln, (hf, vf) in zip(self.lines, warm):
                ln.HF, ln.VF = hf, vf
        n = 6 * nb
        K = np.zeros([n, n])
        J = np.zeros([2 * len(self.lines), n])
        for i in range(n):
            h = dx if i % 6 < 3 else dth
            out = []
            for sgn in (1.0, -1.0):
                Xs = [x.copy() for x in X0]
                Xs[i // 6][i % 6] += sgn * h
                restore()
                self.set_body_positions(Xs)
                out.append((self.coupled_forces(lines_only=True), self.tensions()))
            K[:, i] = -(out[0][0] - out[1][0]) / (2 * h)
            J[:, i] = (out[0][1] - out[1][1]) / (2 * h)
        restore()
        for b, x in zip(self.bodies, X0):
            b.set_position(x)
        self._solve_lines()
        restore()                  # back to the exact state on entry (lines re-solved from it)
        self._solve_lines()
        return (K, J) if tensions else K


def _isnum(s):
    try:
        float(s)
        return True
    except ValueError:
        return False
