"""FOWT: one floating wind turbine's frequency-domain hydrodynamics on the device.

Mirrors the hot-path surface of the reference class (raft/raft_fowt.py): same method names,
argument meaning, return values and the side-effect attributes downstream code reads
(SURVEY.md §8(b)).  The per-node / per-bin arithmetic runs in librafthip; this class owns
the per-design preparation (members, node tables, linear matrices) and the device buffers.

The statics (member inertia / hydrostatics / RNA) are computed on
the host by raft/statics.py, the mooring by raft/mooring.py, and an operating rotor's
aero-servo coefficients by raft/rotor.py (its blade-element solve is CCBlade's, a dependency of
the reference that has to be installed for wind > 0).  Not built here: BEM
(pyHAMS), BEM coefficient files (potFirstOrder=1) and underwater rotors.  External .12d QTFs
(potSecOrder=2) are read on the host (qtf_io.read_qtf12d) and applied on the device
(rh_force_2nd).
"""
import os
import ctypes

import numpy as np

from . import _native as N
from .hydro_math import DEG2RAD, alternator, get_from_dict, wave_numbers, translate_matrix_6to6
from .member import Member
from .rotor import Rotor
from .statics import RNA, fowt_statics
from .prep import DeviceDesign

STATICS_KEYS = ["M_struc", "B_struc", "C_struc", "C_hydro", "W_struc", "W_hydro"]
# turbine inputs a full Rotor (aerodynamics and control, raft/rotor.py) needs
AERO_KEYS = ("blade", "airfoils", "wt_ops", "pitch_control", "torque_control", "gear_ratio", "I_drivetrain",
             "nBlades", "Rhub", "precone")


def transform_force(f_in, offset):
    """transformForce with an offset only (raft/helpers.py:404-452): a force (and moment) at
    `offset` as force and moment about the origin."""
    f = np.array(f_in) if len(f_in) == 6 else np.hstack([f_in, [0, 0, 0]])
    f[3:] += np.cross(offset, f[:3])
    return f


class _Zeros:
    """Pickle stand-in for a large all-zero array (the per-bin aero/BEM matrices of a design
    without them): host preparation in worker processes ships ~70 KB per design, not ~1.4 MB."""

    def __init__(self, a):
        self.shape, self.dtype = a.shape, a.dtype


class FOWT:
    def __getstate__(self):
        st = dict(self.__dict__)
        st["_dd"] = None          # device buffers never travel (host tables do)
        for k, v in st.items():
            if isinstance(v, np.ndarray) and v.size > 4096 and not v.any():
                st[k] = _Zeros(v)
        return st

    def __setstate__(self, st):
        self.__dict__.update({k: np.zeros(v.shape, v.dtype) if isinstance(v, _Zeros) else v for k, v in st.items()})

    def __init__(self, design, w, mpb=None, depth=600, x_ref=0, y_ref=0, heading_adjust=0, device=0):
        self.nDOF = 6
        self.w = np.array(w, dtype=float)
        self.nw = len(self.w)
        self.dw = self.w[1] - self.w[0]
        self.depth = float(depth)
        self.x_ref, self.y_ref = x_ref, y_ref
        self.heading_adjust = heading_adjust
        self.r6 = np.zeros(6)
        self.Xi0 = np.zeros(6)
        self.Xi = np.zeros([self.nDOF, self.nw], dtype=complex)
        self.device_index = device
        self.k = wave_numbers(self.w, self.depth)          # raft/raft_fowt.py:113
        site = design["site"]
        self.rho_water = get_from_dict(site, "rho_water", default=1025.0)
        self.g = get_from_dict(site, "g", default=9.81)
        plat = design["platform"]
        self.potModMaster = get_from_dict(plat, "potModMaster", dtype=int, default=0)
        dlsMax = get_from_dict(plat, "dlsMax", default=5.0)
        self.memberList = []
        self.nplatmems = 0                 # raft/raft_fowt.py:61-67
        self.ntowers = 0
        self.rnaList = []                  # RNA inertia/pose per rotor (raft/statics.py)
        for mi in plat["members"]:
            self.nplatmems += len(mi["heading"]) if "heading" in mi else 1
            mi = dict(mi)
            if self.potModMaster in [1]:
                mi["potMod"] = False
            elif self.potModMaster in [2, 3]:
                mi["potMod"] = True
            if "dlsMax" not in mi:
                mi["dlsMax"] = dlsMax
            headings = get_from_dict(mi, "heading", shape=-1, default=0.)
            for hd in np.atleast_1d(headings):
                self.memberList.append(Member(mi, self.nw, heading=float(hd) + heading_adjust))
        self.nrotors = 0
        self._rotor_submerged = False
        self._aero_mod = []
        turb = design.get("turbine")
        if turb:
            self.nrotors = get_from_dict(turb, "nrotors", dtype=int, shape=0, default=1)
            towers = turb.get("tower")
            if towers is not None:
                towers = towers if isinstance(towers, list) else [towers] * self.nrotors
                self.ntowers = len(towers)
                for mem in towers:
                    self.memberList.append(Member(mem, self.nw))
            nac = turb.get("nacelle")
            if nac is not None:
                for mem in (nac if isinstance(nac, list) else [nac] * self.nrotors):
                    self.memberList.append(Member(mem, self.nw))
            tcopy = dict(turb)
            tcopy["nrotors"] = self.nrotors
            hhub = np.atleast_1d(get_from_dict(turb, "hHub", shape=-1, default=100.0))
            self._rotor_submerged = bool(np.any(hhub < 0))
            if all(k in tcopy for k in ("mRNA", "IxRNA", "IrRNA", "xCG_RNA", "overhang", "shaft_tilt")):
                if not self._rotor_submerged and all(k in tcopy for k in AERO_KEYS):
                    # full rotors (raft/rotor.py): the site's fluid properties are copied into
                    # the turbine inputs as raft/raft_fowt.py:85-90 does
                    for k, dflt in (("rho_air", 1.225), ("mu_air", 1.81e-05), ("shearExp_air", 0.12),
                                    ("rho_water", 1025.0), ("mu_water", 1.0e-03), ("shearExp_water", 0.12)):
                        tcopy[k] = get_from_dict(site, k, shape=0, default=dflt)
                    self.rnaList = [Rotor(tcopy, self.w, ir) for ir in range(self.nrotors)]
                else:
                    self.rnaList = [RNA(tcopy, ir, get_from_dict) for ir in range(self.nrotors)]
            self._aero_mod = np.atleast_1d(get_from_dict(turb, "aeroServoMod", shape=-1, default=1))
        self.potSecOrder = get_from_dict(plat, "potSecOrder", dtype=int, default=0)
        if self.potSecOrder == 1:
            mn, mx = plat["min_freq2nd"], plat["max_freq2nd"]
            df = plat.get("df_freq2nd", mn)
            self.w1_2nd = np.arange(mn, mx + 0.5 * mn, df) * 2 * np.pi   # raft/raft_fowt.py:240
            self.w2_2nd = self.w1_2nd.copy()
            self.k1_2nd = wave_numbers(self.w1_2nd, self.depth)
            self.k2_2nd = self.k1_2nd.copy()
        elif self.potSecOrder == 2:                                       # raft/raft_fowt.py:248-252
            if "hydroPath" not in plat:
                raise Exception("If potSecOrder==2, then hydroPath must be specified in the platform input.")
            self.qtfPath = plat["hydroPath"] + ".12d"
            self.readQTF(self.qtfPath)
        self.outFolderQTF = plat.get("outFolderQTF")
        self.C_moor = np.zeros([6, 6])
        self.F_moor0 = np.zeros(6)
        self.body = mpb                    # this FOWT's body in an array-level mooring system
        # this FOWT's own mooring system (raft/raft_fowt.py:166-189; MoorPy there, raft/mooring.py here)
        self.ms = None
        moor = design.get("mooring")
        if moor:
            from .mooring import MooringSystem
            self.ms = MooringSystem.from_yaml(moor)
            self.ms.transform(trans=[x_ref, y_ref], rot=heading_adjust)
            self.ms.initialize()
        self.yawstiff = plat.get("yaw_stiffness", 0)                     # :194-197
        self.shearExp_water = get_from_dict(site, "shearExp_water", default=0.12)   # :117
        self.D_hydro = np.zeros(6)
        self.f_aero0 = np.zeros([6, self.nrotors])
        self.A_BEM = np.zeros([6, 6, self.nw])
        self.B_BEM = np.zeros([6, 6, self.nw])
        self.A_hydro_morison = np.zeros([6, 6])
        self.B_gyro = np.zeros([6, 6, max(self.nrotors, 1)])
        self.A_aero = np.zeros([6, 6, self.nw, self.nrotors])
        self.B_aero = np.zeros([6, 6, self.nw, self.nrotors])
        self.f_aero = np.zeros([6, self.nw, self.nrotors], dtype=complex)
        self._statics = None
        for k in ("M_struc", "B_struc", "C_struc", "C_hydro"):
            setattr(self, k, np.zeros([6, 6]))   # filled by calcStatics
        self._dd = None            # DeviceDesign (built lazily, invalidated on setPosition)
        self._host = None          # its host-side tables (prep.host_tables), same lifetime
        self._qtf_devs = {}        # QtfDevice per heading (same lifetime as _dd)
        self.nWaves = 1

    # ------------------------------------------------------------------ set-up
    @property
    def rotorList(self):
        """The reference's name for the rotors (raft/raft_fowt.py:201): Rotor objects when the
        turbine carries its aerodynamic inputs, else their RNA pose/inertia part."""
        return self.rnaList

    def setPosition(self, r6):
        """raft/raft_fowt.py:260-288: members, rotors and this FOWT's mooring system; the
        mooring stiffness C_moor and mean force F_moor0 follow the new pose (unless a C_moor
        was given to setStatics)."""
        self.r6 = np.array(r6, dtype=float)
        self.Xi0 = self.r6 - np.array([self.x_ref, self.y_ref, 0, 0, 0, 0])
        for mem in self.memberList:
            mem.setPosition(r6=self.r6)
        for rot in self.rnaList:
            rot.setPosition(self.r6)
        if self.ms is not None:
            self.ms.set_body_positions([self.r6])
            self.F_moor0 = self.ms.body_forces(self.ms.bodies[0], lines_only=True)
            if "C_moor" not in (self._statics or {}):
                self.C_moor = self.ms.coupled_stiffness_analytic()
        self._dd = self._host = None
        self._qtf_devs = {}

    def setStatics(self, statics):
        """Override calcStatics with given matrices (M_struc, B_struc, C_struc, C_hydro, ...)
        and optionally C_moor -- e.g. the reference's own values for a regression run, or a
        mooring stiffness from an external MoorPy model."""
        self._statics = {k: np.array(v, dtype=float) for k, v in statics.items()}

    def calcStatics(self):
        """raft/raft_fowt.py:291-565: member inertia and hydrostatics summed about the PRP
        (raft/statics.py).  Matrices given to setStatics() override the computed ones (a
        full set skips the computation), and its C_moor stands in for MoorPy's stiffness."""
        given = self._statics or {}
        full = all(k in given for k in ("M_struc", "C_struc", "C_hydro"))
        computable = not self._rotor_submerged and (self.nrotors == 0 or len(self.rnaList) == self.nrotors)
        if not full and not computable:
            if self._rotor_submerged:
                raise NotImplementedError("underwater rotors (blade-member buoyancy, raft/raft_fowt.py:386-443) "
                                          "are outside the accelerated path")
            raise ValueError("turbine: mRNA, IxRNA, IrRNA, xCG_RNA, overhang and shaft_tilt are required")
        if computable:
            # also when a full set is given: the tower masses and member inertias feed the
            # tower-base channels of saveTurbineOutputs (raft/raft_fowt.py:1939-1970)
            fowt_statics(self)
        self._dd = self._host = None
        if self._statics is None:
            return
        for k in STATICS_KEYS:
            if k in self._statics:
                setattr(self, k, self._statics[k].copy())
        if "B_struc" not in self._statics:
            self.B_struc = np.zeros([6, 6])
        if "C_moor" in self._statics:
            self.C_moor = self._statics["C_moor"].copy()
        self._dd = self._host = None

    def calcCurrentLoads(self, case):
        """Mean Morison drag of a uniform current with a power-law depth profile on every
        submerged strip node, as forces and moments about the PRP (raft/raft_fowt.py:1297-1382).
        Host arithmetic: 6 numbers per design and case, outside the response solve."""
        rho = self.rho_water
        D = np.zeros(6)
        speed = get_from_dict(case, "current_speed", shape=0, default=0.0)
        heading = get_from_dict(case, "current_heading", shape=0, default=0)
        Zref = 0.0
        for rot in self.rnaList:
            if rot.r3[2] < 0:
                Zref = rot.r3[2]
        ch, sh = np.cos(np.deg2rad(heading)), np.sin(np.deg2rad(heading))
        for mem in self.memberList:
            circ = mem.shape == "circular"
            for il in range(mem.ns):
                if not (mem.r[il, 2] < 0):
                    continue
                v = speed * ((self.depth - abs(mem.r[il, 2])) / (self.depth + Zref)) ** self.shearExp_water
                vrel = np.array([v * ch, v * sh, 0])
                vq = np.sum(vrel * mem.q) * mem.q
                vp = vrel - vq
                vp1 = np.sum(vrel * mem.p1) * mem.p1
                vp2 = np.sum(vrel * mem.p2) * mem.p2
                ds, drs, dls = mem.ds[il], mem.drs[il], mem.dls[il]
                if circ:
                    aq, ap1, ap2 = np.pi * ds * dls, ds * dls, ds * dls
                    aend = np.abs(np.pi * ds * drs)
                    n1 = n2 = np.linalg.norm(vp)
                else:
                    aq = 2 * (ds[0] + ds[0]) * dls
                    ap1, ap2 = ds[0] * dls, ds[1] * dls
                    aend = np.abs((ds[0] + drs[0]) * (ds[1] + drs[1]) - (ds[0] - drs[0]) * (ds[1] - drs[1]))
                    n1, n2 = np.linalg.norm(vp1), np.linalg.norm(vp2)
                nq = np.linalg.norm(vq)
                Dq = 0.5 * rho * aq * mem.coef("Cd_q", il) * nq * vq
                Dp1 = 0.5 * rho * ap1 * mem.coef("Cd_p1", il) * n1 * vp1
                Dp2 = 0.5 * rho * ap2 * mem.coef("Cd_p2", il) * n2 * vp2
                Dend = 0.5 * rho * aend * mem.coef("Cd_End", il) * nq * vq
                f = Dq + Dp1 + Dp2 + Dend
                r = mem.r[il, :] - self.r6[:3]
                D[:3] += f
                D[3:] += np.cross(r, f)
        self.D_hydro = D
        return D

    def calcTurbineConstants(self, case, ptfm_pitch=0):
        """raft/raft_fowt.py:773-845: for every operating rotor with aeroServoMod > 0 at wind
        speed > 0, the aero-servo added mass, damping and wind excitation of Rotor.calcAero
        (raft/rotor.py; CCBlade evaluates the blades) moved from the hub to the platform
        reference point (translateMatrix6to6DOF / transformForce with r_hub_rel), the mean aero
        loads f_aero0 and the rotor's gyroscopic damping B_gyro.  Host work: 6x6 per bin."""
        status = get_from_dict(case, "turbine_status", shape=0, dtype=str, default="operating")
        had_aero = bool(np.any(self.A_aero) or np.any(self.B_aero) or np.any(self.B_gyro))
        self.A_aero = np.zeros([6, 6, self.nw, self.nrotors])
        self.B_aero = np.zeros([6, 6, self.nw, self.nrotors])
        self.f_aero = np.zeros([6, self.nw, self.nrotors], dtype=complex)
        self.f_aero0 = np.zeros([6, self.nrotors])
        self.B_gyro = np.zeros([6, 6, max(self.nrotors, 1)])
        if self._rotor_submerged:
            raise NotImplementedError("underwater rotors (raft/raft_rotor.py) are outside the accelerated path")
        if status == "operating":
            speed = get_from_dict(case, "wind_speed", shape=0, default=10.0)
            mods = np.atleast_1d(self._aero_mod)
            for ir in range(self.nrotors):
                rot = self.rnaList[ir] if ir < len(self.rnaList) else None
                mod = rot.aeroServoMod if isinstance(rot, Rotor) else mods[min(ir, len(mods) - 1)]
                if not (mod > 0 and speed > 0.0):
                    continue
                if not isinstance(rot, Rotor):
                    raise NotImplementedError("rotor aerodynamics need the turbine's blade, airfoil, operating-point "
                                              "and control inputs (raft/raft_rotor.py:37-374)")
                f0, f, a, b = rot.calcAero(case)
                for iw in range(self.nw):
                    self.A_aero[:, :, iw, ir] = translate_matrix_6to6(a[:, :, iw], rot.r_hub_rel)
                    self.B_aero[:, :, iw, ir] = translate_matrix_6to6(b[:, :, iw], rot.r_hub_rel)
                    self.f_aero[:, iw, ir] = transform_force(f[:, iw], rot.r_hub_rel)
                self.f_aero0[:, ir] = transform_force(f0, rot.r_hub_rel)
                Omega_rpm = np.interp(speed, rot.Uhub, rot.Omega_rpm)
                IO_rotor = rot.I_drivetrain * (rot.q * Omega_rpm * 2 * np.pi / 60)
                self.B_gyro[3:, 3:, ir] = alternator(IO_rotor)
        if had_aero or np.any(self.A_aero) or np.any(self.B_aero) or np.any(self.B_gyro):
            self._dd = self._host = None          # the per-bin M and B of the device design change

    def calcHydroConstants(self):
        """raft/raft_fowt.py:848-880 (strip-theory members)."""
        self.A_hydro_morison = np.zeros([6, 6])
        for mem in self.memberList:
            k_array = self.k if mem.MCF else None
            self.A_hydro_morison += mem.calcHydroConstants(r_ref=self.r6[:3], rho=self.rho_water, g=self.g,
                                                           k_array=k_array)
        self._dd = self._host = None
        self._qtf_devs = {}

    def host_tables(self):
        """Host-side node/member tables and linear matrices of the current pose and
        coefficients (prep.host_tables; cached, and carried along when the FOWT is pickled)."""
        if self._host is None:
            from .prep import host_tables
            self._host = host_tables(self)
        return self._host

    def device_design(self):
        """The DeviceDesign of the current pose and coefficients (built on first use)."""
        if self._dd is None:
            self._dd = DeviceDesign(self, device=self.device_index)
        return self._dd

    # ------------------------------------------------------------------ sea state
    def _sea_state(self, case):
        """raft/raft_fowt.py:982-1014: normalises `case` in place (tiled arrays), returns
        heading [deg], spectrum codes, Hs, Tp, gamma per sea state."""
        hd = case["wave_heading"]
        self.nWaves = 1 if np.isscalar(hd) else len(hd)
        nW = self.nWaves
        case["wave_heading"] = get_from_dict(case, "wave_heading", shape=nW, dtype=float, default=0)
        case["wave_spectrum"] = get_from_dict(case, "wave_spectrum", shape=nW, dtype=str, default="JONSWAP")
        case["wave_period"] = get_from_dict(case, "wave_period", shape=nW, dtype=float)
        case["wave_height"] = get_from_dict(case, "wave_height", shape=nW, dtype=float)
        case["wave_gamma"] = get_from_dict(case, "wave_gamma", shape=nW, dtype=float, default=0)
        for sp in case["wave_spectrum"]:
            if sp not in N.SPECTRUM_CODES:
                raise ValueError(f"Wave spectrum input '{sp}' not recognized.")
        self.beta = case["wave_heading"] * DEG2RAD
        return (np.array(case["wave_heading"], dtype=float), [N.SPECTRUM_CODES[s] for s in case["wave_spectrum"]],
                np.array(case["wave_height"], dtype=float), np.array(case["wave_period"], dtype=float),
                np.array(case["wave_gamma"], dtype=float))

    def calcHydroExcitation(self, case, memberList=[], dgamma=0):
        """Sea state + strip-theory inertial excitation (raft/raft_fowt.py:972-1149) on the
        device.  Sets beta, S, zeta, F_hydro_iner [nWaves,6,nw], F_BEM and the per-member
        kinematics mem.u/ud/pDyn like the reference."""
        import torch
        dd = self.device_design()
        hd, spec, Hs, Tp, gam = self._sea_state(case)
        nW = self.nWaves
        heads = dd.ensure_headings(hd * DEG2RAD)
        dev = dd.device
        f64 = dict(dtype=torch.float64, device=dev)
        S = torch.empty([nW, self.nw], **f64)
        zeta = torch.empty([nW, self.nw], **f64)
        spec_t = torch.tensor(spec, dtype=torch.int32, device=dev)
        Hs_t, Tp_t, g_t = (torch.tensor(x, **f64) for x in (Hs, Tp, gam))
        N.check(N.lib().rh_sea_state(N.context(dd.dev_index), nW, self.nw, N.ptr(dd.w), float(self.dw), N.ptr(spec_t),
                                     N.ptr(Hs_t), N.ptr(Tp_t), N.ptr(g_t), N.ptr(S), N.ptr(zeta),
                                     N.stream_handle(torch, dev)), "rh_sea_state")
        hidx = torch.tensor(heads, dtype=torch.long, device=dev)
        F = dd.finer.index_select(0, hidx) * zeta[:, None, :]
        self._zeta_dev = zeta
        self._S_dev = S
        self._heads = heads
        self.S = S.cpu().numpy()
        self.zeta = zeta.cpu().numpy().astype(complex)
        self.F_hydro_iner = F.cpu().numpy()
        self.F_BEM = np.zeros([nW, 6, self.nw], dtype=complex)
        self._fill_member_kinematics(memberList, dd, heads, zeta)

    def _fill_member_kinematics(self, memberList, dd, heads, zeta):
        """mem.u / ud / pDyn side effects (raft/raft_fowt.py:1021-1024,1108-1110)."""
        if not memberList:
            return
        U = (dd.uhat.index_select(0, dd.torch.tensor(heads, dtype=dd.torch.long, device=dd.device))
             * zeta[:, None, None, :]).cpu().numpy()
        w = self.w
        j = 0
        for mem in self.memberList:
            mem.u = np.zeros([self.nWaves, mem.ns, 3, self.nw], dtype=complex)
            mem.ud = np.zeros_like(mem.u)
            for il in range(mem.ns):
                if mem.r[il, 2] < 0:
                    mem.u[:, il] = U[:, j]
                    mem.ud[:, il] = 1j * w * U[:, j]
                    j += 1

    # ------------------------------------------------------------------ drag
    def calcHydroLinearization(self, Xi):
        """Borgman drag linearisation for the response Xi [6,nw] (raft/raft_fowt.py:1152-1266):
        returns B_hydro_drag [6,6]; sets mem.Bmat, self.F_hydro_drag (sea state 0)."""
        import torch
        dd = self.device_design()
        if getattr(self, "_zeta_dev", None) is None:
            raise RuntimeError("calcHydroExcitation must be called first (wave kinematics)")
        dev = dd.device
        Xi_t = torch.tensor(np.asarray(Xi, dtype=complex), dtype=torch.complex128, device=dev).contiguous()
        B = torch.empty(36, dtype=torch.float64, device=dev)
        Bm = torch.zeros([max(dd.nn, 1), 9], dtype=torch.float64, device=dev)
        F = torch.empty([6, self.nw], dtype=torch.complex128, device=dev)
        z0 = self._zeta_dev[0].contiguous()
        d = dd.struct()
        N.check(N.lib().rh_linearize(N.context(dd.dev_index), ctypes.byref(d), int(self._heads[0]), N.ptr(Xi_t),
                                     N.ptr(z0), N.ptr(B), N.ptr(Bm), N.ptr(F), N.stream_handle(torch, dev)),
                "rh_linearize")
        self._Bmat_dev = Bm
        self.B_hydro_drag = B.reshape(6, 6).cpu().numpy()
        self.F_hydro_drag = F.cpu().numpy()
        self._scatter_bmat(Bm.cpu().numpy())
        return self.B_hydro_drag

    def _scatter_bmat(self, bm):
        j = 0
        for mem in self.memberList:
            mem.Bmat = np.zeros([mem.ns, 3, 3])
            for il in range(mem.ns):
                if mem.r[il, 2] < 0:
                    mem.Bmat[il] = bm[j].reshape(3, 3)
                    j += 1

    def calcDragExcitation(self, ih):
        """raft/raft_fowt.py:1270-1293"""
        import torch
        dd = self.device_design()
        dev = dd.device
        F = torch.empty([6, self.nw], dtype=torch.complex128, device=dev)
        d = dd.struct()
        z = self._zeta_dev[ih].contiguous()
        N.check(N.lib().rh_drag_excitation(N.context(dd.dev_index), ctypes.byref(d), int(self._heads[ih]), N.ptr(z),
                                           N.ptr(self._Bmat_dev), N.ptr(F), N.stream_handle(torch, dev)),
                "rh_drag_excitation")
        self.F_hydro_drag = F.cpu().numpy()
        return self.F_hydro_drag

    # ------------------------------------------------------------------ second order
    def _qtf_device(self, beta):
        from .qtf import QtfDevice
        key = (float(beta), np.asarray(self.w1_2nd, dtype=float).tobytes(), np.asarray(self.k1_2nd, dtype=float).tobytes())
        if key not in self._qtf_devs:
            self._qtf_devs[key] = QtfDevice(self, self.w1_2nd, self.k1_2nd, float(beta), self.device_index)
        return self._qtf_devs[key]

    def calcQTF_slenderBody(self, waveHeadInd, Xi0=None, verbose=False, iCase=None, iWT=None):
        """Slender-body QTF of the body for heading self.beta[waveHeadInd]
        (raft/raft_fowt.py:1385-1645) computed by rh_qtf_slender.  Xi0: motion RAOs [6, nw]
        (numpy or device tensor; None = fixed body).  Sets self.qtf [n2, n2, 1, 6] and
        self.heads_2nd; with outFolderQTF and verbose, writes the .4 / .12d files."""
        import torch
        if getattr(self, "w1_2nd", None) is None:
            raise RuntimeError("calcQTF_slenderBody needs potSecOrder=1 (min_freq2nd/max_freq2nd)")
        dd = self.device_design()
        beta = float(self.beta[waveHeadInd])
        self.heads_2nd = [beta]
        if waveHeadInd not in (0, -1):
            # the reference's qtf has one heading and is indexed with waveHeadInd
            # (raft/raft_fowt.py:1442, 1456): every other sea state raises
            from .second_order import qtf_index_error
            raise qtf_index_error(waveHeadInd)
        qd = self._qtf_device(beta)
        if Xi0 is None:
            X = torch.zeros([6, self.nw], dtype=torch.complex128, device=dd.device)
        elif isinstance(Xi0, torch.Tensor):
            X = Xi0.to(device=dd.device, dtype=torch.complex128).contiguous()
        else:
            X = torch.tensor(np.asarray(Xi0, dtype=complex), dtype=torch.complex128, device=dd.device)
        M66 = torch.tensor(np.asarray(self.M_struc, dtype=float), dtype=torch.float64, device=dd.device).contiguous()
        if verbose:
            print(f" Computing QTF for heading {beta:.2f}")
        q = qd.qtf(dd.w, X, M66)
        self._qtf_dev, self._qtf_qd = q, qd
        self.qtf = q.cpu().numpy()[:, :, None, :]
        if self.outFolderQTF is not None and verbose:
            from .qtf_io import write_rao4, qtf_file_names
            rao_path, qtf_path = qtf_file_names(self.outFolderQTF, beta, iCase, iWT)
            Xi_2nd = np.array([np.interp(self.w1_2nd, self.w, x, left=0, right=0) for x in X.cpu().numpy()])
            write_rao4(rao_path, self.w1_2nd, beta, Xi_2nd)
            self.writeQTF(self.qtf, qtf_path)

    def readQTF(self, flPath, ULEN=1):
        """WAMIT .12d reader (raft/raft_fowt.py:1651-1697): sets heads_2nd [rad], w1_2nd,
        w2_2nd and qtf [n1, n2, nheads, 6]."""
        from .qtf_io import read_qtf12d
        self.heads_2nd, self.w1_2nd, self.w2_2nd, self.qtf = read_qtf12d(flPath, self.rho_water, self.g, ULEN,
                                                                          self.nDOF)
        self._qtf_file_dev = {}     # device copies per heading (calcHydroForce_2ndOrd)

    def _file_qtf_device(self, beta):
        """The file QTF at heading beta as the device operands of rh_force_2nd.  Heading
        interpolation as raft/raft_fowt.py:1752-1757 does it, fill values included."""
        import torch
        from types import SimpleNamespace
        key = float(beta)
        if key not in self._qtf_file_dev:
            h2 = np.asarray(self.heads_2nd, dtype=float)
            if len(h2) == 1:
                qb = self.qtf[:, :, 0, :]
            else:
                from scipy.interpolate import interp1d
                q = self.qtf
                re = interp1d(h2, q, assume_sorted=True, axis=2, bounds_error=False,
                              fill_value=(q[:, :, 0, :], q[:, :, -1, :].real))(beta)
                im = interp1d(h2, q, assume_sorted=True, axis=2, bounds_error=False,
                              fill_value=(q[:, :, 0, :], q[:, :, -1, :].imag))(beta)
                qb = re + 1j * im
            dev = torch.device("cuda", self.device_index)
            w2 = torch.tensor(np.asarray(self.w1_2nd, dtype=float), dtype=torch.float64, device=dev)
            qd = SimpleNamespace(torch=torch, dev=dev, dev_index=self.device_index, n2=len(self.w1_2nd), w2=w2)
            qt = torch.tensor(np.ascontiguousarray(qb, dtype=complex), dtype=torch.complex128, device=dev).contiguous()
            self._qtf_file_dev[key] = (qd, qt)
        return self._qtf_file_dev[key]

    def writeQTF(self, qtfIn, outPath, w=None):
        """WAMIT .12d writer (raft/raft_fowt.py:1700-1726)."""
        from .qtf_io import write_qtf12d
        w1 = self.w1_2nd if w is None else w
        write_qtf12d(outPath, qtfIn, w1, self.heads_2nd, self.rho_water, self.g)

    def calcHydroForce_2ndOrd(self, beta, S0, iCase=None, iWT=None, interpMode="qtf"):
        """Difference-frequency force amplitudes and mean drift from the QTF
        (raft/raft_fowt.py:1728-1818) on the device.  interpMode 'qtf' (the default: the QTF
        resampled to (w, w), then the force spectrum) or 'spectrum' (the force spectrum on the
        QTF grid, then resampled; f is complex with zero imaginary part, as the reference's).
        Returns (f_mean [6], f [6, nw]) like the reference."""
        import torch
        if interpMode not in ("qtf", "spectrum"):
            raise ValueError(f"calcHydroForce_2ndOrd: interpMode must be 'qtf' or 'spectrum', not {interpMode!r}")
        h2 = getattr(self, "heads_2nd", None)
        from_file = self.potSecOrder == 2
        if h2 is None or (not from_file and getattr(self, "_qtf_dev", None) is None):
            raise RuntimeError("calcHydroForce_2ndOrd needs a QTF (calcQTF_slenderBody or a .12d file)")
        if beta < h2[0]:
            print(f"Warning in calcHydroForce_2ndOrd: angle {beta} is less than the minimum incidence angle in the "
                  f"QTF. An incidence of {h2[0]} will be considered for 2nd order loads.")
        if beta > h2[-1]:
            print(f"Warning in calcHydroForce_2ndOrd: angle {beta} is more than the maximum incidence angle in the "
                  f"QTF. An incidence of {h2[-1]} will be considered for 2nd order loads.")
        from .qtf import force_2nd, force_2nd_spectrum
        dd = self.device_design()
        qd, qt = self._file_qtf_device(beta) if from_file else (self._qtf_qd, self._qtf_dev)
        S = S0 if isinstance(S0, torch.Tensor) else torch.tensor(np.asarray(S0, dtype=float), dtype=torch.float64,
                                                                  device=dd.device)
        kern = force_2nd if interpMode == "qtf" else force_2nd_spectrum
        fm, f = kern(qd, qt, dd.w, self.dw, S.to(dd.device).contiguous())
        self._f2nd_dev = f
        f_mean, f_h = fm.cpu().numpy(), f.cpu().numpy()
        if self.outFolderQTF is not None:
            from .qtf_io import write_f2nd
            write_f2nd(os.path.join(self.outFolderQTF, f"f_2nd-_Case{iCase + 1}_WT{iWT}.txt"), self.w, f_h)
        return f_mean, f_h

    # ------------------------------------------------------------------ outputs
    def rotor_channels(self):
        """Coefficient rows of the derived rotor channels for rh_channel_stats and their mean
        values (raft/raft_fowt.py:1900-1970 with zero aero loads: A_aero = B_aero = f_aero0 = 0,
        the only state the accelerated path runs).  Per rotor ir:
          AxRNA_ir = w^2 (Xi_surge + zHub Xi_pitch)                              (:1909-1913)
          Mbase_ir = m hArm w^2 Xi_surge + (w^2 (m hArm zCG + I_CG) + m g hArm) Xi_pitch
        (M_I + M_w of :1947-1960 expanded).  Returns (coef [2 nrot, 2, 6], means [2 nrot])."""
        nr = self.nrotors
        coef = np.zeros([2 * nr, 2, 6])
        means = np.zeros(2 * nr)
        for ir, rot in enumerate(self.rnaList):
            coef[ir, 1, 0] = 1.0
            coef[ir, 1, 4] = rot.r_rel[2]
            means[ir] = abs(np.sin(self.Xi0[4]) * 9.81)                              # :1914
        for ir, rot in enumerate(self.rnaList[:len(self.mtower)]):
            mt = self.mtower[ir] + rot.mRNA
            zCG = (self.rCG_tow[ir][2] * self.mtower[ir] + rot.r_rel[2] * rot.mRNA) / mt
            tower = self.memberList[self.nplatmems + ir]
            hArm = zCG - tower.rA[2]
            ICG = (translate_matrix_6to6(tower.M_struc, [0, 0, -zCG])[4, 4] + rot.mRNA * (rot.r_rel[2] - zCG) ** 2
                   + rot.IrRNA)
            k = nr + ir
            coef[k, 0, 4] = mt * self.g * hArm
            coef[k, 1, 0] = mt * hArm
            coef[k, 1, 4] = mt * hArm * zCG + ICG
            means[k] = mt * self.g * hArm * np.sin(self.Xi0[4])                      # :1965-1966, f_aero0 = 0
        return coef, means

    def _aero_outputs(self, results, case):
        """The channels operating rotors change (host arithmetic over nw values per rotor):
        the tower-base moment with the aero reaction term and the mean thrust moment
        (raft/raft_fowt.py:1950-1970), and the rotor azimuth / speed / torque / pitch response
        through the control transfer function C of Rotor.calcAero (:1976-2045)."""
        rms = lambda x: np.sqrt(0.5 * np.sum(np.abs(x) ** 2))                      # getRMS
        psd = lambda x: np.sum(0.5 * np.abs(x) ** 2 / self.dw, axis=0)              # getPSD, 2-D
        w, Xi = self.w, self.Xi
        for ir, rot in enumerate(self.rnaList[:len(self.mtower)]):
            if not (np.any(self.A_aero[..., ir]) or np.any(self.B_aero[..., ir]) or np.any(self.f_aero0[:, ir])):
                continue
            mt = self.mtower[ir] + rot.mRNA
            zCG = (self.rCG_tow[ir][2] * self.mtower[ir] + rot.r_rel[2] * rot.mRNA) / mt
            tower = self.memberList[self.nplatmems + ir]
            zBase = tower.rA[2]
            hArm = zCG - zBase
            ICG = (translate_matrix_6to6(tower.M_struc, [0, 0, -zCG])[4, 4] + rot.mRNA * (rot.r_rel[2] - zCG) ** 2
                   + rot.IrRNA)
            aCG = -w ** 2 * (Xi[:, 0, :] + zCG * Xi[:, 4, :])
            M_I = -mt * aCG * hArm - ICG * (-w ** 2 * Xi[:, 4, :])
            M_w = mt * self.g * hArm * Xi[:, 4]
            M_X = -(-w ** 2 * self.A_aero[0, 0, :, ir] + 1j * w * self.B_aero[0, 0, :, ir]) * (rot.r_rel[2] - zBase) ** 2 \
                * Xi[:, 4, :]
            dyn = M_I + M_w + 0.0 + M_X
            avg = mt * self.g * hArm * np.sin(self.Xi0[4]) + transform_force(self.f_aero0[:, ir], [0, 0, -hArm])[4]
            results["Mbase_avg"][ir] = avg
            results["Mbase_std"][ir] = rms(dyn)
            results["Mbase_PSD"][:, ir] = psd(dyn)
            results["Mbase_max"][ir] = avg + 3 * results["Mbase_std"][ir]
            results["Mbase_min"][ir] = avg - 3 * results["Mbase_std"][ir]
        speed = get_from_dict(case, "wind_speed", shape=0, default=10.0)
        for ir, rot in enumerate(self.rnaList):
            if not (isinstance(rot, Rotor) and rot.aeroServoMod > 1 and speed > 0.0 and hasattr(rot, "C")):
                continue
            XiHub = Xi[:, 0, :] + rot.r_rel[2] * Xi[:, 4, :]
            phi = np.zeros_like(XiHub, dtype=complex)
            for ih in range(Xi.shape[0] - 1):
                phi[ih] = rot.C * XiHub[ih]
            phi[-1] = rot.C * (XiHub[-1] - rot.V_w / (1j * w))
            omega_w = 1j * w * phi
            torque_w = (1j * w * rot.kp_tau + rot.ki_tau) * phi
            pitch_w = (1j * w * rot.kp_beta + rot.ki_beta) * phi
            rpm = lambda x: x / 0.1047                                                  # radps2rpm (helpers.py:32)
            results["omega_avg"][ir] = rot.Omega_case
            results["omega_std"][ir] = rpm(rms(omega_w))
            results["omega_max"][ir] = results["omega_avg"][ir] + 2 * results["omega_std"][ir]
            results["omega_min"][ir] = results["omega_avg"][ir] - 2 * results["omega_std"][ir]
            results["omega_PSD"][:, ir] = rpm(1) ** 2 * psd(omega_w)
            results["torque_avg"][ir] = rot.aero_torque / rot.Ng
            results["torque_std"][ir] = rms(torque_w)
            results["torque_PSD"][:, ir] = psd(torque_w)
            results["power_avg"][ir] = rot.aero_power
            results["bPitch_avg"][ir] = rot.pitch_case
            results["bPitch_std"][ir] = rms(pitch_w) * 57.29577951308232
            results["bPitch_PSD"][:, ir] = 57.29577951308232 ** 2 * psd(pitch_w)
            results["wind_PSD"] = 0.5 * np.abs(rot.V_w) ** 2 / self.dw

    def saveTurbineOutputs(self, results, case):
        """raft/raft_fowt.py:1821-2045: platform motions (RMS, PSD, RA), nacelle acceleration
        AxRNA_* and tower-base moment Mbase_* per rotor (rh_channel_stats on the device; with an
        operating rotor the aero reaction term and mean thrust moment are added on the host,
        _aero_outputs) and wave_PSD.  Rotor-control channels (omega/torque/power/bPitch,
        wind_PSD) come from the rotor's control transfer function when aeroServoMod > 1 and the
        wind blows, else they are the reference's zeros.  Mooring tensions (Tmoor_*) need a
        mooring system (raft/mooring.py; MoorPy in the reference)."""
        import torch
        self.Xi0 = self.r6 - np.array([self.x_ref, self.y_ref, 0, 0, 0, 0])
        stats = getattr(self, "_stats", None)
        if stats is None:
            raise RuntimeError("saveTurbineOutputs needs the device motion statistics of solveDynamics")
        for i, dof in enumerate(["surge", "sway", "heave", "roll", "pitch", "yaw"]):
            conv = 57.29577951308232 if i >= 3 else 1.0
            avg = self.Xi0[i] * conv
            std = stats["std"][i]
            results[f"{dof}_avg"] = avg
            results[f"{dof}_std"] = std
            results[f"{dof}_max"] = avg + 3 * std
            results[f"{dof}_min"] = avg - 3 * std
            results[f"{dof}_PSD"] = stats["psd"][i]
            results[f"{dof}_RA"] = self.Xi[:, i, :] * conv
        nr = self.nrotors
        coef, means = self.rotor_channels()
        psd = np.zeros([2 * nr, self.nw])
        std = np.zeros(2 * nr)
        if nr > 0:
            X = self._xi_dev
            dev = X.device
            ct = torch.tensor(coef, dtype=torch.float64, device=dev).contiguous()
            wt = torch.tensor(self.w, dtype=torch.float64, device=dev)
            pt = torch.empty([2 * nr, self.nw], dtype=torch.float64, device=dev)
            stt = torch.empty([2 * nr], dtype=torch.float64, device=dev)
            N.check(N.lib().rh_channel_stats(N.context(self.device_index), 1, X.shape[0], 6, self.nw, float(self.dw),
                                             N.ptr(wt), N.ptr(X), 2 * nr, N.ptr(ct), N.ptr(pt), N.ptr(stt),
                                             N.stream_handle(torch, dev)), "rh_channel_stats")
            psd, std = pt.cpu().numpy(), stt.cpu().numpy()
        for j, name in enumerate(["AxRNA", "Mbase"]):
            sl = slice(j * nr, (j + 1) * nr)
            results[f"{name}_std"] = std[sl].copy()
            results[f"{name}_PSD"] = psd[sl].T.copy()                                 # [nw, nrotors]
            results[f"{name}_avg"] = means[sl].copy()
            results[f"{name}_max"] = means[sl] + 3 * std[sl]
            results[f"{name}_min"] = means[sl] - 3 * std[sl]
        results["wave_PSD"] = np.sum(0.5 * np.abs(self.zeta) ** 2 / self.dw, axis=0)
        for name in ["omega_avg", "omega_std", "omega_max", "omega_min", "torque_avg", "torque_std", "power_avg",
                     "bPitch_avg", "bPitch_std"]:                                     # :1983-1994
            results[name] = np.zeros(nr)
        for name in ["omega_PSD", "torque_PSD", "bPitch_PSD"]:
            results[name] = np.zeros([self.nw, nr])
        self._aero_outputs(results, case)
        if self.ms is not None and self.ms.lines:                                      # :1878-1898
            results.update(mooring_outputs(self.ms, self._xi_dev, self.w, self.device_index, self._xi_dev.shape[0]))


def mooring_outputs(ms, X, w, device, nrow):
    """Mooring-tension channels (raft/raft_fowt.py:1878-1898, raft/raft_model.py:346-388):
    mean end tensions T = getTensions(), tension amplitudes J_moor Xi with the central-
    difference tension Jacobian (getCoupledStiffness(tensions=True)), their RMS and PSD
    (rh_channel_stats; the reference divides this PSD by w[0] instead of dw)."""
    import torch
    T = ms.tensions()
    _, J = ms.coupled_stiffness_fd(tensions=True)
    nT, ndof = J.shape
    dev = X.device
    coef = np.zeros([nT, 2, ndof])
    coef[:, 0, :] = J
    ct = torch.tensor(coef, dtype=torch.float64, device=dev).contiguous()
    wt = torch.tensor(np.asarray(w, dtype=float), dtype=torch.float64, device=dev)
    pt = torch.empty([nT, len(w)], dtype=torch.float64, device=dev)
    st = torch.empty([nT], dtype=torch.float64, device=dev)
    N.check(N.lib().rh_channel_stats(N.context(device), 1, int(nrow), int(ndof), len(w), float(w[0]), N.ptr(wt),
                                     N.ptr(X.contiguous()), nT, N.ptr(ct), N.ptr(pt), N.ptr(st),
                                     N.stream_handle(torch, dev)), "rh_channel_stats")
    std = st.cpu().numpy()
    return {"Tmoor_avg": T, "Tmoor_std": std, "Tmoor_max": T + 3 * std, "Tmoor_min": T - 3 * std,
            "Tmoor_PSD": pt.cpu().numpy()}
