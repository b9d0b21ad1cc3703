"""Rotor aerodynamics and control linearisation (raft/raft_rotor.py).

What the frequency-domain solve consumes from an operating rotor at wind > 0: the mean hub
loads f0, the aero-servo added mass a(w) and damping b(w), and the wind excitation f(w), all
about the hub in global orientation (Rotor.calcAero, raft/raft_rotor.py:788-1005), plus the
rotor-averaged turbulence spectrum they are driven by (IECKaimal, :1125-1250).

The blade-element momentum solve itself is CCBlade's (Rotor.runCCBlade, :699-768), a
third-party dependency of the reference (raft/raft_rotor.py:17-20, WISDEM/CCBlade).  It is
imported the same way here and built with the same inputs: the blade stations, chord, twist,
precurve/presweep and the airfoil polars resampled on the reference's angle-of-attack grid and
spline-interpolated over the span by relative thickness (:178-331).  Where CCBlade is not
installed (this image), a Rotor still builds every input, and calcAero raises unless a
CCBlade-compatible object is attached as `rotor.ccblade` (the parity tests attach a scripted
one; tests/golden/make_golden.py golden_rotor runs the reference with the same script).

Host code: per (case, rotor) it is a handful of 6x6 matrices per frequency bin; the device
solve takes the result as per-bin mass and damping (raft/prep.py linear_matrices).
"""
import numpy as np
from scipy.interpolate import PchipInterpolator
from scipy.special import iv, modstruve

from .hydro_math import get_from_dict, rotation_matrix
from .statics import RNA

# the reference's own truncated unit constants (raft/raft_rotor.py:31-32), kept: the gain
# schedule angles and the CCBlade derivative conversions are computed with them
RAD2DEG = 57.2958
RPM2RADPS = 0.1047


def ccblade_classes():
    """(CCBlade, CCAirfoil) from the installed package, as raft/raft_rotor.py:17-20 imports
    them, else the restatement in raft/ccblade.py (Ning's BEM as CCBlade implements it,
    pinned by the reference's wind-case expectations)."""
    try:
        from ccblade.ccblade import CCBlade, CCAirfoil
        return CCBlade, CCAirfoil
    except ImportError:
        try:
            from wisdem.ccblade.ccblade import CCBlade, CCAirfoil
            return CCBlade, CCAirfoil
        except ImportError:
            from .ccblade import CCAirfoil, CCBlade
            return CCBlade, CCAirfoil


class IECWind:
    """The IEC 61400-1 turbulence parameters RAFT uses (raft/pyIECWind.py:8-77): turbine class
    -> V_ref, turbulence category -> I_ref, and the NTM / ETM / EWM standard deviations."""

    def __init__(self):
        self.Turbine_Class = "I"
        self.Turbulence_Class = "B"
        self.z_hub = 90.0

    def setup(self):
        self.V_ref = {"I": 50.0, "II": 42.5, "III": 37.5, "IV": 30.0}.get(self.Turbine_Class, getattr(self, "V_ref", None))
        if self.V_ref is not None:
            self.V_ave = self.V_ref * 0.2
        ref = {"A+": 0.18, "A": 0.16, "B": 0.14, "C": 0.12}
        if self.Turbulence_Class in ref:
            self.I_ref = ref[self.Turbulence_Class]
        self.Sigma_1 = 42 if self.z_hub > 60 else 0.7 * self.z_hub

    def NTM(self, V_hub):
        return self.I_ref * (0.75 * V_hub + 5.6)

    def ETM(self, V_hub):
        c = 2
        return c * self.I_ref * (0.072 * (self.V_ave / c + 3) * (V_hub / c - 4) + 10)

    def EWM(self, V_hub):
        V_e50 = 1.4 * self.V_ref
        return 0.11 * V_hub, V_e50, 0.8 * V_e50, self.V_ref, 0.8 * self.V_ref


def _rotate6(M, R):
    """rotateMatrix6 (raft/helpers.py:507-542) of a [6, 6] or [6, 6, n] tensor."""
    out = np.zeros_like(M)
    if M.ndim == 2:
        out[:3, :3] = R @ M[:3, :3] @ R.T
        out[:3, 3:] = R @ M[:3, 3:] @ R.T
        out[3:, :3] = out[:3, 3:].T
        out[3:, 3:] = R @ M[3:, 3:] @ R.T
        return out
    for i in range(M.shape[2]):
        out[:, :, i] = _rotate6(M[:, :, i], R)
    return out


class Rotor(RNA):
    """One rotor of a FOWT: the RNA pose of raft/statics.py plus the aerodynamic inputs,
    operating schedule, control gains and the aero-servo linearisation of raft/raft_rotor.py.

    turbine : the design's turbine dict with the site entries FOWT copies into it
              (rho_air, mu_air, shearExp_air, rho_water, mu_water, shearExp_water;
              raft/raft_fowt.py:85-90)
    w       : frequencies [rad/s];  ir : rotor index
    ccblade : optional (CCBlade, CCAirfoil) classes; default: the installed package."""

    def __init__(self, turbine, w, ir, ccblade=None):
        nr = turbine["nrotors"]
        get = get_from_dict
        self.w = np.array(w)
        self.nw = len(self.w)
        self.turbine = turbine
        self.ir = ir
        self.platform_heading = 0.0
        self.R_ptfm = np.eye(3)
        RNA.__init__(self, turbine, ir, get)                         # :46-113 pose inputs
        self.speed_gain = get(turbine, "speed_gain", shape=nr, default=1.0)[ir]
        self.nBlades = get(turbine, "nBlades", shape=nr, dtype=int)[ir]
        self.azimuths = get(turbine, "headings", shape=-1, default=list(np.arange(self.nBlades) * 360. / self.nBlades))
        self.Rhub = get(turbine, "Rhub", shape=nr)[ir]
        self.precone = get(turbine, "precone", shape=nr)[ir]
        self.aeroServoMod = get(turbine, "aeroServoMod", shape=nr, default=1)[ir]
        self.q_rel = rotation_matrix(0, self.shaft_tilt, self.shaft_toe) @ np.array([1., 0., 0.])
        self.hHub = self.r_rel[2] + self.q_rel[2] * self.overhang
        self.Zhub = self.hHub
        self.setPosition(np.zeros(6))

        if isinstance(turbine["blade"], dict):
            turbine["blade"] = [turbine["blade"]] * nr
        if isinstance(turbine["wt_ops"], dict):
            turbine["wt_ops"] = [turbine["wt_ops"]] * nr
        blade = turbine["blade"][ir]
        self.R_rot = get(blade, "Rtip", shape=-1)
        for b in turbine["blade"]:                                     # :139-153
            r0, rtip_b = b["geometry"][0][0], b["geometry"][-1][0]
            if not (r0 >= self.Rhub and rtip_b <= self.R_rot):
                raise ValueError(f"Input blade geometry is invalid. First node radius needs to be >= Rhub ({self.Rhub}) "
                                 f"or last node radius needs to be <= Rtip ({self.R_rot})")
        ops = turbine["wt_ops"][ir]
        Uhub = get(ops, "v", shape=-1)
        self.I_drivetrain = get(turbine, "I_drivetrain", shape=nr)[ir]
        # operating schedule, parked above 1.4 x cut-out (:161-164)
        self.Uhub = np.r_[Uhub, Uhub.max() * 1.4, 100]
        self.Omega_rpm = np.r_[get(ops, "omega_op", shape=-1), 0, 0]
        self.pitch_deg = np.r_[get(ops, "pitch_op", shape=-1), 90, 90]
        self.kp_0 = np.zeros_like(self.Uhub)
        self.ki_0 = np.zeros_like(self.Uhub)
        self.k_float = 0
        self.f0 = np.zeros(6)
        self._airfoils(turbine, blade, get)
        if self.r3[2] < 0:                                              # :315-323
            self.rho, self.mu, self.shearExp = turbine["rho_water"], turbine["mu_water"], turbine["shearExp_water"]
        else:
            self.rho, self.mu, self.shearExp = turbine["rho_air"], turbine["mu_air"], turbine["shearExp_air"]
        self.nSector = get(blade, "nSector", default=4)
        self.precurveTip, self.presweepTip = blade["precurveTip"], blade["presweepTip"]
        self.ccblade = None
        cls, af_cls = ccblade if ccblade is not None else ccblade_classes()
        if cls is not None:
            self.ccblade = self.build_ccblade(cls, af_cls)
        self.setControlGains(turbine)
        if self.r3[2] + self.R_rot < 0:
            raise NotImplementedError("underwater rotors (blade members, raft/raft_rotor.py:522-637) are outside the "
                                      "accelerated path")

    # ------------------------------------------------------------------ CCBlade inputs
    def _airfoils(self, turbine, blade, get):
        """The polar and blade tables handed to CCBlade (raft/raft_rotor.py:178-313): each
        airfoil's cl/cd/cm (and cpmin) on a 200-point angle-of-attack grid, made periodic at
        +-180 deg; per blade element the polars and added-mass coefficients spline-interpolated
        (PCHIP) by relative thickness over nr equal span elements; chord, twist, precurve and
        presweep interpolated at the element radii."""
        st_af = [b for a, b in blade["airfoils"]]
        st_pos = [a for a, b in blade["airfoils"]]
        n_aoa = 200
        aoa = np.unique(np.hstack([np.linspace(-180, -30, int(n_aoa / 4.0 + 1)), np.linspace(-30, 30, int(n_aoa / 2.0)),
                                   np.linspace(30, 180, int(n_aoa / 4.0 + 1))]))
        afs = turbine["airfoils"]
        n_af = len(afs)
        names = [a["name"] for a in afs]
        thick = np.array([a["relative_thickness"] for a in afs], dtype=float)
        Ca = np.array([a.get("added_mass_coeff", [0.5, 1.0]) for a in afs], dtype=float).reshape(n_af, 2)
        cl = np.zeros((n_af, n_aoa, 1))
        cd = np.zeros((n_af, n_aoa, 1))
        cm = np.zeros((n_af, n_aoa, 1))
        cpmin = np.zeros((n_af, n_aoa, 1))
        cpmin_flag = len(np.array(afs[-1]["data"])[0]) > 4             # decided on the last airfoil (:207-210)
        for i in range(n_af):
            tab = np.array(afs[i]["data"])
            cl[i, :, 0] = np.interp(aoa, tab[:, 0], tab[:, 1])
            cd[i, :, 0] = np.interp(aoa, tab[:, 0], tab[:, 2])
            cm[i, :, 0] = np.interp(aoa, tab[:, 0], tab[:, 3])
            if cpmin_flag:
                cpmin[i, :, 0] = np.interp(aoa, tab[:, 0], tab[:, 4])
            for arr in ((cl, cd, cm, cpmin) if cpmin_flag else (cl, cd, cm)):
                if abs(arr[i, 0, 0] - arr[i, -1, 0]) > 1.0e-5:
                    arr[i, 0, 0] = arr[i, -1, 0]
        nr = get(blade, "nr", default=20)
        grid = np.linspace(0., 1., nr, endpoint=False) + 0.5 / nr
        ns = len(st_af)
        st_thick = np.zeros(ns)
        st_Ca = np.zeros((ns, 2))
        st_cl, st_cd, st_cm, st_cp = (np.zeros((ns, n_aoa, 1)) for _ in range(4))
        for i in range(ns):
            if st_af[i] in names:                                         # first match (:258-268)
                j = names.index(st_af[i])
                st_thick[i], st_Ca[i] = thick[j], Ca[j]
                st_cl[i], st_cd[i], st_cm[i], st_cp[i] = cl[j], cd[j], cm[j], cpmin[j]
        if not np.all(st_thick == np.flip(sorted(st_thick))):
            raise NotImplementedError("airfoils not ordered thickest to thinnest from root to tip (the reference "
                                      "stops in a debugger there, raft/raft_rotor.py:296-303)")
        self.r_thick_interp = PchipInterpolator(st_pos, st_thick)(grid)
        thick_u, idx = np.unique(st_thick, return_index=True)
        self.Ca_interp = PchipInterpolator(st_pos, st_Ca)(grid)
        flip = np.flip(self.r_thick_interp)
        self.cl_interp = np.flip(PchipInterpolator(thick_u, st_cl[idx, :, :])(flip), axis=0)
        self.cd_interp = np.flip(PchipInterpolator(thick_u, st_cd[idx, :, :])(flip), axis=0)
        self.cm_interp = np.flip(PchipInterpolator(thick_u, st_cm[idx, :, :])(flip), axis=0)
        self.cpmin_interp = np.flip(PchipInterpolator(thick_u, st_cp[idx, :, :])(flip), axis=0)
        self.aoa = aoa
        geo = np.array(blade["geometry"])
        rtip = turbine["blade"][-1]["geometry"][-1][0]     # the last blade type's, as the reference's loop leaves it
        self.dr = (rtip - self.Rhub) / nr
        self.blade_r = np.linspace(self.Rhub, rtip, nr, endpoint=False) + self.dr / 2
        self.blade_chord = np.interp(self.blade_r, geo[:, 0], geo[:, 1])
        self.blade_theta = np.interp(self.blade_r, geo[:, 0], geo[:, 2])
        self.blade_precurve = np.interp(self.blade_r, geo[:, 0], geo[:, 3])
        self.blade_presweep = np.interp(self.blade_r, geo[:, 0], geo[:, 4])

    def build_ccblade(self, CCBlade, CCAirfoil):
        """A CCBlade object with the reference's arguments (raft/raft_rotor.py:331-370)."""
        af = [CCAirfoil(self.aoa, [], self.cl_interp[i, :, :], self.cd_interp[i, :, :], self.cm_interp[i, :, :])
              for i in range(self.cl_interp.shape[0])]
        blade = self.turbine["blade"][self.ir]
        return CCBlade(self.blade_r, self.blade_chord, self.blade_theta, af, self.Rhub, blade["Rtip"], self.nBlades,
                       self.rho, self.mu, self.precone, np.degrees(self.shaft_tilt), 0.0, self.shearExp, self.r3[2],
                       self.nSector, self.blade_precurve, self.precurveTip, self.blade_presweep, self.presweepTip,
                       tiploss=True, hubloss=True, wakerotation=True, usecd=True, derivatives=True)

    # ------------------------------------------------------------------ pose
    def setPosition(self, r6=np.zeros(6), R=None):
        """raft/raft_rotor.py:376-409."""
        r6 = np.asarray(r6, dtype=float)
        self.R_ptfm = np.array(R) if R is not None else rotation_matrix(*r6[3:])
        self.platform_heading = r6[5]
        self.setYaw()
        self.r_RRP_rel = self.R_ptfm @ self.r_rel
        self.r_CG_rel = self.r_RRP_rel + self.q * self.xCG_RNA
        self.r_hub_rel = self.r_RRP_rel + self.q * self.overhang
        self.r3 = r6[:3] + self.r_hub_rel

    def setYaw(self, yaw=None):
        """raft/raft_rotor.py:412-458."""
        if yaw is not None:
            self.yaw_command = np.radians(yaw)
        if self.yaw_mode == 0:
            self.yaw = self.inflow_heading - self.platform_heading + self.yaw_command
        elif self.yaw_mode == 1:
            self.yaw = self.turbine_heading - self.platform_heading
        elif self.yaw_mode == 2:
            self.yaw = self.yaw_command
        elif self.yaw_mode == 3:
            self.yaw = self.yaw_command - self.platform_heading
        else:
            raise Exception('Unsupported yaw_mode value. Must be 0, 1, or 2.')
        self.turbine_heading = self.platform_heading + self.yaw
        R_q_rel = rotation_matrix(0, self.shaft_tilt, self.shaft_toe + self.yaw)
        self.R_q = R_q_rel @ self.R_ptfm
        self.q_rel = R_q_rel @ np.array([1, 0, 0])
        self.q = self.R_ptfm @ self.q_rel
        return self.yaw

    # ------------------------------------------------------------------ control
    def setControlGains(self, turbine):
        """ROSCO gains, sign-flipped (raft/raft_rotor.py:770-785)."""
        pc = turbine["pitch_control"]
        ang = np.array(pc["GS_Angles"]) * RAD2DEG
        self.kp_0 = np.interp(self.pitch_deg, ang, pc["GS_Kp"], left=0, right=0)
        self.ki_0 = np.interp(self.pitch_deg, ang, pc["GS_Ki"], left=0, right=0)
        self.k_float = -pc["Fl_Kp"]
        self.kp_tau = -turbine["torque_control"]["VS_KP"]
        self.ki_tau = -turbine["torque_control"]["VS_KI"]
        self.Ng = turbine["gear_ratio"]

    # ------------------------------------------------------------------ aerodynamics
    def runCCBlade(self, U0, tilt=0, yaw_misalign=0):
        """One CCBlade evaluation at the scheduled operating point (raft/raft_rotor.py:699-768)."""
        if self.ccblade is None:
            raise NotImplementedError("rotor aerodynamics need CCBlade (a dependency of the reference, "
                                      "raft/raft_rotor.py:17-20), which is not installed; attach a CCBlade-compatible "
                                      "object as rotor.ccblade")
        Uhub = U0 * self.speed_gain
        Omega_rpm = np.interp(Uhub, self.Uhub, self.Omega_rpm)
        pitch_deg = np.interp(Uhub, self.Uhub, self.pitch_deg)
        self.ccblade.tilt = tilt
        self.ccblade.yaw = yaw_misalign
        loads, derivs = self.ccblade.evaluate(Uhub, Omega_rpm, pitch_deg, coefficients=True)
        self.U_case, self.Omega_case, self.pitch_case = Uhub, Omega_rpm, pitch_deg
        self.aero_torque, self.aero_power, self.aero_thrust = loads["Q"][0], loads["P"][0], loads["T"][0]
        J = {("P", "r"): derivs["dP"]["dr"]}
        for k in ("Q", "T"):
            d = derivs["d" + k]
            J[k, "Uhub"] = np.atleast_1d(np.diag(d["dUinf"]))
            J[k, "pitch_deg"] = np.atleast_1d(np.diag(d["dpitch"]))
            J[k, "Omega_rpm"] = np.atleast_1d(np.diag(d["dOmega"]))
        self.J = J
        return loads, derivs

    def calcAero(self, case, current=False, display=0):
        """Mean hub loads f0 [6], wind excitation f [6, nw], aero-servo added mass a and damping
        b [6, 6, nw] about the hub in global orientation (raft/raft_rotor.py:788-1005):
        aeroServoMod 1 = thrust-speed derivative only; 2 = with the pitch / torque PI control
        loop closed through the drivetrain."""
        if current:
            raise NotImplementedError("underwater rotors (current-driven) are outside the accelerated path")
        self.a = np.zeros([6, 6, self.nw])
        self.b = np.zeros([6, 6, self.nw])
        self.f = np.zeros([6, self.nw], dtype=complex)
        self.f0 = np.zeros(6)
        speed = get_from_dict(case, "wind_speed", shape=0, default=10)
        heading = get_from_dict(case, "wind_heading", shape=0, default=0.0)
        self.inflow_heading = np.radians(heading)
        self.turbine_heading = np.radians(get_from_dict(case, "turbine_heading", shape=0, default=0.0))
        self.setYaw()
        yaw_misalign = np.arctan2(self.q[1], self.q[0]) - self.inflow_heading
        turbine_tilt = np.arctan2(self.q[2], np.hypot(self.q[0], self.q[1]))
        loads, derivs = self.runCCBlade(speed, tilt=turbine_tilt, yaw_misalign=yaw_misalign)
        dT_dU = np.atleast_1d(np.diag(derivs["dT"]["dUinf"]))
        dT_dOm = np.atleast_1d(np.diag(derivs["dT"]["dOmega"])) / RPM2RADPS
        dT_dPi = np.atleast_1d(np.diag(derivs["dT"]["dpitch"])) * RAD2DEG
        dQ_dU = np.atleast_1d(np.diag(derivs["dQ"]["dUinf"]))
        dQ_dOm = np.atleast_1d(np.diag(derivs["dQ"]["dOmega"])) / RPM2RADPS
        dQ_dPi = np.atleast_1d(np.diag(derivs["dQ"]["dpitch"])) * RAD2DEG
        forces_axis = np.array([loads["T"][0], loads["Y"][0], loads["Z"][0]])
        moments_axis = np.array([loads["My"][0], loads["Q"][0], loads["Mz"][0]])
        self.f0[:3] = self.R_q @ forces_axis
        self.f0[3:] = self.R_q @ moments_axis
        _, _, _, S_rot = self.IECKaimal(case, current=current)
        self.V_w = np.array(np.sqrt(S_rot), dtype=complex)
        w = self.w
        if self.aeroServoMod == 1:
            b_in = np.zeros([6, 6, self.nw])
            b_in[0, 0, :] = dT_dU
            f_in = np.zeros([6, self.nw], dtype=complex)
            f_in[0, :] = dT_dU * self.V_w
            self.a = _rotate6(np.zeros([6, 6, self.nw]), self.R_q)
            self.b = _rotate6(b_in, self.R_q)
            self.f[:3, :] = self.R_q @ f_in[:3, :]
        elif self.aeroServoMod == 2:
            self.kp_beta = -np.interp(speed, self.Uhub, self.kp_0)
            self.ki_beta = -np.interp(speed, self.Uhub, self.ki_0)
            kp_tau = self.kp_tau * (self.kp_beta == 0)
            ki_tau = self.ki_tau * (self.ki_beta == 0)
            # drivetrain / control transfer functions per bin (:900-930), as arrays over w
            D = self.I_drivetrain * w ** 2 + (dQ_dOm + self.kp_beta * dQ_dPi - self.Ng * kp_tau) * 1j * w \
                + self.ki_beta * dQ_dPi - self.Ng * ki_tau
            self.C = 1j * w * (dQ_dU - self.k_float * dQ_dPi / self.r3[2]) / D
            H_QT = ((dT_dOm + self.kp_beta * dT_dPi) * 1j * w + self.ki_beta * dT_dPi) / (
                self.I_drivetrain * w ** 2 + (dQ_dOm + self.kp_beta * dQ_dPi - self.Ng * kp_tau) * 1j * w
                + self.ki_beta * dQ_dPi - self.Ng * ki_tau)
            self.c_exc = dT_dU - H_QT * dQ_dU
            f2 = (dT_dU - H_QT * dQ_dU) * self.V_w
            b2 = np.real(dT_dU - self.k_float * dT_dPi - H_QT * (dQ_dU - self.k_float * dQ_dPi))
            a2 = np.real((dT_dU - self.k_float * dT_dPi - H_QT * (dQ_dU - self.k_float * dQ_dPi)) / (1j * w))
            R = self.R_q
            for iw in range(self.nw):
                self.a[:3, :3, iw] = R @ np.diag([a2[iw], 0, 0]) @ R.T
                self.b[:3, :3, iw] = R @ np.diag([b2[iw], 0, 0]) @ R.T
                self.f[:3, iw] = R @ np.array([f2[iw], 0, 0])
        return self.f0, self.f, self.a, self.b

    def IECKaimal(self, case, current=False):
        """Rotor-averaged Kaimal wind spectrum (raft/raft_rotor.py:1125-1250): IEC 61400-1
        turbulence from a class string ('IB_NTM') or an intensity, Kaimal u/v/w spectra, and
        the rotor-averaged longitudinal spectrum.  Returns (U, V, W, Rot) [(m/s)^2/Hz]."""
        if current:
            speed = get_from_dict(case, "current_speed", shape=0, default=1.0)
            turbulence = get_from_dict(case, "current_turbulence", shape=0, default=0.0, dtype=str)
        else:
            speed = get_from_dict(case, "wind_speed", shape=0, default=10.0)
            turbulence = get_from_dict(case, "turbulence", shape=0, default=0.0, dtype=str)
        f = self.w / 2 / np.pi
        HH = abs(self.r3[2])
        R = self.R_rot
        V_ref = speed
        iec = IECWind()
        iec.z_hub = HH
        TurbMod = None
        if isinstance(turbulence, str):
            Class = ""
            char = ""
            for char in turbulence:
                if char == "I" or char == "V":
                    Class += char
                else:
                    break
            if not Class:
                Class = "I"
                try:
                    turbulence = float(turbulence)
                except ValueError:
                    raise Exception(f"Turbulence class must start with I, II, III, or IV: case['turbulence'] = {turbulence}")
            else:
                iec.Turbulence_Class = char
                try:
                    TurbMod = turbulence.split("_")[1]
                except IndexError:
                    raise Exception(f"Error reading the turbulence model: {turbulence}")
            iec.Turbine_Class = Class
        iec.setup()
        if isinstance(turbulence, int):
            turbulence = float(turbulence)
        if isinstance(turbulence, float):
            iec.I_ref = turbulence
            TurbMod = "NTM"
        if TurbMod == "NTM":
            sigma_1 = iec.NTM(V_ref)
        elif TurbMod == "ETM":
            sigma_1 = iec.ETM(V_ref)
        elif TurbMod == "EWM":
            sigma_1 = iec.EWM(V_ref)[0]
        else:
            raise Exception("Wind model must be either NTM, ETM, or EWM. While you wrote " + str(TurbMod))
        L_1 = .7 * HH if HH <= 60 else 42.
        sigma_u, L_u = sigma_1, 8.1 * L_1
        sigma_v, L_v = 0.8 * sigma_1, 2.7 * L_1
        sigma_w, L_w = 0.5 * sigma_1, 0.66 * L_1
        U = (4 * L_u / V_ref) * sigma_u ** 2 / ((1 + 6 * f * L_u / V_ref) ** (5. / 3.))
        V = (4 * L_v / V_ref) * sigma_v ** 2 / ((1 + 6 * f * L_v / V_ref) ** (5. / 3.))
        W = (4 * L_w / V_ref) * sigma_w ** 2 / ((1 + 6 * f * L_w / V_ref) ** (5. / 3.))
        kappa = 12 * np.sqrt((f / V_ref) ** 2 + (0.12 / L_u) ** 2)
        Rot = (2 * U / (R * kappa) ** 3) * \
            (modstruve(1, 2 * R * kappa) - iv(1, 2 * R * kappa) - 2 / np.pi
             + R * kappa * (-2 * modstruve(-2, 2 * R * kappa) + 2 * iv(2, 2 * R * kappa) + 1))
        Rot[np.isnan(Rot)] = 0
        return U, V, W, Rot
