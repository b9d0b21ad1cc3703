"""Strip-theory member: discretisation, pose and per-node hydrodynamic constants.

Per-design host preparation feeding the device node tables:
  * strip discretisation         raft/raft_member.py:169-220
  * pose (q, p1, p2, node r)     raft/raft_member.py:245-304
  * added mass / inertial coeffs raft/raft_member.py:877-1050
  * MacCamy-Fuchs Cm             raft/raft_member.py:1053-1088
The member statics (getInertia / getHydrostatics, §8(f) row 1) are computed from these
tables by raft/statics.py (and natively by csrc/rh_prep.h for design sweeps).
"""
import numpy as np
from scipy.special import hankel1

from .hydro_math import get_from_dict, rotation_matrix, translate_matrix_3to6


class Member:
    def __init__(self, mi, nw, heading=0.0):
        self.name = str(mi["name"])
        self.type = int(mi["type"])
        rA0 = np.array(mi["rA"], dtype=float)
        rB0 = np.array(mi["rB"], dtype=float)
        if (rA0[2] == 0 or rB0[2] == 0) and self.type != 3:
            raise ValueError("RAFT Members cannot start or end on the waterplane")
        if rB0[2] < rA0[2]:          # end A must be the lower end (raft/raft_member.py:41-44)
            rA0, rB0 = rB0, rA0
        shape = str(mi["shape"])
        self.potMod = get_from_dict(mi, "potMod", dtype=bool, default=False)
        self.MCF = get_from_dict(mi, "MCF", dtype=bool, default=False)
        self.gamma = get_from_dict(mi, "gamma", default=0.0)
        rAB = rB0 - rA0
        self.l = np.linalg.norm(rAB)
        if heading != 0.0:           # rotated copies about z (raft/raft_member.py:56-64)
            c, s = np.cos(np.deg2rad(heading)), np.sin(np.deg2rad(heading))
            rot = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])
            rA0 = rot @ rA0
            rB0 = rot @ rB0
            if rAB[0] == 0.0 and rAB[1] == 0:
                self.gamma += heading
        self.rA0, self.rB0 = rA0, rB0

        st = np.array(mi["stations"], dtype=float)
        n = len(st)
        if n < 2:
            raise ValueError("At least two stations entries must be provided")
        if not sorted(st) == st.tolist():
            raise ValueError(f"Member {self.name}: the station list is not in ascending order.")
        self.stations = (st - st[0]) / (st[-1] - st[0]) * self.l

        if shape[0].lower() == "c":
            self.shape = "circular"
            self.d = get_from_dict(mi, "d", shape=n)
            self.gamma = 0
        elif shape[0].lower() == "r":
            self.shape = "rectangular"
            self.sl = get_from_dict(mi, "d", shape=[n, 2])
        else:
            raise ValueError("The only allowable shape strings are circular and rectangular")
        if self.MCF and self.shape != "circular":
            self.MCF = False

        # shell, ballast and caps for the statics (raft/raft_member.py:99-154, used by
        # raft/statics.py); `t` is required there, so its absence only fails calcStatics
        self.t = get_from_dict(mi, "t", shape=n) if "t" in mi else None
        self.rho_shell = get_from_dict(mi, "rho_shell", shape=0, default=8500.)
        st_fill = get_from_dict(mi, "l_fill", shape=n - 1, default=0)
        for i in range(n - 1):
            if st_fill[i] < 0:
                raise Exception(f"Member {self.name}: ballast level in section {i+1} is negative.")
            if st_fill[i] > st[i + 1] - st[i]:
                raise Exception(f"Member {self.name}: ballast level in section {i+1} exceeds section length."
                                + f" ({st_fill[i]} > {st[i+1] - st[i]}).")
        self.l_fill = st_fill / (st[-1] - st[0]) * self.l
        rho_fill = get_from_dict(mi, "rho_fill", shape=-1, default=1025)
        if np.isscalar(rho_fill):
            self.rho_fill = np.zeros(n - 1) + rho_fill
        elif len(rho_fill) == n - 1:
            self.rho_fill = np.array(rho_fill)
        else:
            raise Exception(f"Member {self.name}: the number of provided ballast densities (rho_fill) must be 1 "
                            "less than the number of stations.")
        cap_st = np.atleast_1d(get_from_dict(mi, "cap_stations", shape=-1, default=[]))
        if len(cap_st) == 0:
            self.cap_t, self.cap_d_in, self.cap_stations = [], [], []
        else:
            self.cap_t = get_from_dict(mi, "cap_t", shape=cap_st.shape[0])
            self.cap_d_in = get_from_dict(mi, "cap_d_in", shape=cap_st.shape[0])
            self.cap_stations = (cap_st - st[0]) / (st[-1] - st[0]) * self.l

        self.Cd_q = get_from_dict(mi, "Cd_q", shape=n, default=0.0)
        self.Cd_p1 = get_from_dict(mi, "Cd", shape=n, default=0.6, index=0)
        self.Cd_p2 = get_from_dict(mi, "Cd", shape=n, default=0.6, index=1)
        self.Cd_End = get_from_dict(mi, "CdEnd", shape=n, default=0.6)
        self.Ca_q = get_from_dict(mi, "Ca_q", shape=n, default=0.0)
        self.Ca_p1 = get_from_dict(mi, "Ca", shape=n, default=0.97, index=0)
        self.Ca_p2 = get_from_dict(mi, "Ca", shape=n, default=0.97, index=1)
        self.Ca_End = get_from_dict(mi, "CaEnd", shape=n, default=0.6)

        self._discretise(mi)
        self.nw = nw
        self.a_i = np.zeros(self.ns)
        self.Amat = np.zeros([self.ns, 3, 3])
        self.Imat = np.zeros([self.ns, 3, 3])
        self.Imat_MCF = None
        self.Bmat = np.zeros([self.ns, 3, 3])
        self.setPosition(np.zeros(6))

    # -- strip discretisation (raft/raft_member.py:169-220) --------------------------
    def _discretise(self, mi):
        circ = self.shape == "circular"
        dorsl = list(self.d) if circ else list(self.sl)
        dlsMax = float(np.atleast_1d(get_from_dict(mi, "dlsMax", shape=1, default=5))[0])
        ls, dls, ds, drs = [0.0], [0.0], [0.5 * dorsl[0]], [0.5 * dorsl[0]]
        for i in range(1, len(self.stations)):
            lstrip = self.stations[i] - self.stations[i - 1]
            if lstrip > 0.0:
                ns = int(np.ceil(lstrip / dlsMax))
                dlstrip = lstrip / ns
                m = 0.5 * (dorsl[i] - dorsl[i - 1]) / lstrip
                ls += [self.stations[i - 1] + dlstrip * (0.5 + j) for j in range(ns)]
                dls += [dlstrip] * ns
                ds += [dorsl[i - 1] + dlstrip * 2 * m * (0.5 + j) for j in range(ns)]
                drs += [dlstrip * m] * ns
            elif lstrip == 0.0:
                ls += [self.stations[i - 1]]
                dls += [0]
                ds += [0.5 * (dorsl[i - 1] + dorsl[i])]
                drs += [0.5 * (dorsl[i] - dorsl[i - 1])]
        ls += [self.stations[-1]]
        dls += [0.0]
        ds += [0.5 * dorsl[-1]]
        drs += [-0.5 * dorsl[-1]]
        self.ns = len(ls)
        self.ls = np.array(ls, dtype=float)
        self.dls = np.array(dls, dtype=float)
        self.ds = np.array(ds)
        self.drs = np.array(drs)
        self.r = np.zeros([self.ns, 3])

    # -- pose (raft/raft_member.py:245-304) --------------------------------------------
    def setPosition(self, r6=np.zeros(6)):
        r6 = np.asarray(r6, dtype=float)
        rAB = self.rB0 - self.rA0
        q = rAB / np.linalg.norm(rAB)
        beta = np.arctan2(q[1], q[0])
        phi = np.arctan2(np.sqrt(q[0] ** 2 + q[1] ** 2), q[2])
        s1, c1 = np.sin(beta), np.cos(beta)
        s2, c2 = np.sin(phi), np.cos(phi)
        s3, c3 = np.sin(np.deg2rad(self.gamma)), np.cos(np.deg2rad(self.gamma))
        R = np.array([[c1 * c2 * c3 - s1 * s3, -c3 * s1 - c1 * c2 * s3, c1 * s2],
                      [c1 * s3 + c2 * c3 * s1, c1 * c3 - c2 * s1 * s3, s1 * s2],
                      [-c3 * s2, s2 * s3, c2]])
        p1 = R @ np.array([1, 0, 0])
        p2 = np.cross(q, p1)
        Rp = rotation_matrix(*r6[3:])
        self.R = Rp @ R
        self.q, self.p1, self.p2 = Rp @ q, Rp @ p1, Rp @ p2
        self.rA = r6[:3] + Rp @ self.rA0        # MoorPy transformPosition(r, r6)
        self.rB = r6[:3] + Rp @ self.rB0
        rABd = self.rB - self.rA
        for i in range(self.ns):
            self.r[i, :] = self.rA + (self.ls[i] / self.l) * rABd
        self.qMat = np.outer(self.q, self.q)
        self.p1Mat = np.outer(self.p1, self.p1)
        self.p2Mat = np.outer(self.p2, self.p2)

    # -- coefficient interpolation at node il (raft/raft_fowt.py:1191-1194) -------------
    def coef(self, name, il):
        return np.interp(self.ls[il], self.stations, getattr(self, name))

    def _side_volume(self, il):
        if self.shape == "circular":
            v = 0.25 * np.pi * self.ds[il] ** 2 * self.dls[il]
        else:
            v = self.ds[il, 0] * self.ds[il, 1] * self.dls[il]
        if self.r[il, 2] + 0.5 * self.dls[il] > 0:      # partly out of the water
            v = v * (0.5 * self.dls[il] - self.r[il, 2]) / self.dls[il]
        return v

    def _end_volume_area(self, il):
        ds, drs = self.ds[il], self.drs[il]
        if self.shape == "circular":
            v = np.pi / 12.0 * abs((ds + drs) ** 3 - (ds - drs) ** 3)
            a = np.pi * ds * drs
        else:
            v = np.pi / 12.0 * ((np.mean(ds + drs)) ** 3 - (np.mean(ds - drs)) ** 3)
            a = (ds[0] + drs[0]) * (ds[1] + drs[1]) - (ds[0] - drs[0]) * (ds[1] - drs[1])
        return v, a

    # -- MacCamy-Fuchs inertia coefficient (raft/raft_member.py:1053-1088) -------------
    def getCmSides(self, il, k=None):
        Ca_p1, Ca_p2 = self.coef("Ca_p1", il), self.coef("Ca_p2", il)
        Cm_p1_0, Cm_p2_0 = (1. + Ca_p1), (1. + Ca_p2)
        if k is None or not self.MCF:
            return Cm_p1_0, Cm_p2_0
        R = self.ds[il] / 2
        Hp1 = 0.5 * (hankel1(0, k * R) - hankel1(2, k * R))
        Cm = 4j / (np.pi * (k * R) ** 2 * Hp1)
        Tr = np.pi / 5 / R
        ramp = 0.5 * (1 - np.cos(np.pi * (k - 0) / Tr)) if k < Tr else 1
        ramp = 0 if k <= 0 else ramp
        return Cm * ramp + Cm_p1_0 * (1 - ramp), Cm * ramp + Cm_p2_0 * (1 - ramp)

    # -- added mass and inertial excitation matrices (raft/raft_member.py:877-1050) ----
    def calcHydroConstants(self, r_ref=np.zeros(3), rho=1025, g=9.81, k_array=None):
        A_hydro = np.zeros([6, 6])
        mcf = self.MCF and k_array is not None
        if mcf:
            self.Imat_MCF = np.zeros([self.ns, 3, 3, len(k_array)], dtype=complex)
        for il in range(self.ns):
            if not (self.r[il, 2] < 0) or self.potMod:
                continue
            v_side = self._side_volume(il)
            Ca_p1, Ca_p2, Ca_End = self.coef("Ca_p1", il), self.coef("Ca_p2", il), self.coef("Ca_End", il)
            v_end, a_end = self._end_volume_area(il)
            # inertial excitation (calcImat, :1017-1050)
            I_end = rho * v_end * Ca_End * self.qMat
            if mcf:
                for ik, k in enumerate(k_array):
                    c1, c2 = self.getCmSides(il, k=k)
                    self.Imat_MCF[il, :, :, ik] = rho * v_side * (c1 * self.p1Mat + c2 * self.p2Mat) + I_end
            else:
                c1, c2 = self.getCmSides(il, k=None)
                self.Imat[il] = rho * v_side * (c1 * self.p1Mat + c2 * self.p2Mat) + I_end
            # added mass (:925-963)
            self.Amat[il] = rho * v_side * (Ca_p1 * self.p1Mat + Ca_p2 * self.p2Mat) + rho * v_end * Ca_End * self.qMat
            self.a_i[il] = a_end
            A_hydro += translate_matrix_3to6(self.Amat[il], self.r[il] - r_ref[:3])
        return A_hydro
