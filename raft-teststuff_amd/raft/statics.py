"""Per-design statics on the host: member inertia, member hydrostatics and the FOWT totals
(SURVEY.md §8(f) row 1).  These run once per design (or design variant of a sweep), before
any device work, and produce the M_struc / C_struc / C_hydro / W_struc / W_hydro matrices
the response solve assembles Z(w) from.

Restated from the reference's behaviour (file:line cited per function), including its
conventions:
  * frustum volume/centroid with the geometric-mean mid area (raft/helpers.py:36-63);
  * shell = outer frustum minus inner frustum, ballast = inner frustum filled to l_fill;
  * the waterplane diameter/side lengths are interpolated with the two end values in the
    order the reference passes them (raft/raft_member.py:769,775);
  * hydrostatic moments of circular members crossing the waterplane use the inclined-
    cylinder formula of raft/raft_member.py:815.
Pinned by the reference's own goldens (tests/test_member.py, tests/test_fowt.py) and by the
statics of the golden fixtures (tests/test_statics.py).
"""
import numpy as np

from .hydro_math import alternator, rotation_matrix, translate_matrix_6to6


# ----------------------------------------------------------------------------- geometry
def frustum_vcv(dA, dB, H):
    """Volume and centroid height (from end A) of a circular (scalar diameters) or
    rectangular (pairs of side lengths) frustum of height H (raft/helpers.py:36-63)."""
    if np.sum(dA) == 0 and np.sum(dB) == 0:
        return 0.0, 0.0
    if np.isscalar(dA) and np.isscalar(dB):
        a1, a2, am = 0.25 * np.pi * dA ** 2, 0.25 * np.pi * dB ** 2, 0.25 * np.pi * dA * dB
    elif len(dA) == 2 and len(dB) == 2:
        a1, a2 = dA[0] * dA[1], dB[0] * dB[1]
        am = np.sqrt(a1 * a2)
    else:
        raise ValueError("Input types not accepted")
    return (a1 + a2 + am) * H / 3, ((a1 + 2 * am + 3 * a2) / (a1 + am + a2)) * H / 4


def _frustum_moi(dA, dB, H, p):
    """Radial MoI about end A and axial MoI of a solid circular frustum of density p
    (raft/raft_member.py:321-339)."""
    if H == 0:
        return 0.0, 0.0
    r1, r2 = dA / 2, dB / 2
    if dA == dB:
        return (1 / 12) * (p * H * np.pi * r1 ** 2) * (3 * r1 ** 2 + 4 * H ** 2), 0.5 * p * np.pi * H * r1 ** 4
    q5 = (r2 ** 5 - r1 ** 5) / (r2 - r1)
    return ((1 / 20) * p * np.pi * H * q5 + (1 / 30) * p * np.pi * H ** 3 * (r1 ** 2 + 3 * r1 * r2 + 6 * r2 ** 2),
            (1 / 10) * p * np.pi * H * q5)


def _rect_frustum_moi(La, Wa, Lb, Wb, H, p):
    """(Ixx, Iyy, Izz) about end A of a solid rectangular frustum (cuboid, truncated
    pyramid or truncated triangular prism) of density p (raft/raft_member.py:341-402)."""
    if H == 0:
        return 0.0, 0.0, 0.0
    if La == Lb and Wa == Wb:
        M = p * La * Wa * H
        return (1 / 12) * M * (Wa ** 2 + 4 * H ** 2), (1 / 12) * M * (La ** 2 + 4 * H ** 2), (1 / 12) * M * (La ** 2 + Wa ** 2)
    if La != Lb and Wa != Wb:
        dL, dW = Lb - La, Wb - Wa
        x2 = (1 / 12) * p * (dL ** 3 * H * (Wb / 5 + Wa / 20) + dL ** 2 * La * H * (3 * Wb / 4 + Wa / 4)
                             + dL * La ** 2 * H * (Wb + Wa / 2) + La ** 3 * H * (Wb / 2 + Wa / 2))
        y2 = (1 / 12) * p * (dW ** 3 * H * (Lb / 5 + La / 20) + dW ** 2 * Wa * H * (3 * Lb / 4 + La / 4)
                             + dW * Wa ** 2 * H * (Lb + La / 2) + Wa ** 3 * H * (Lb / 2 + La / 2))
        z2 = p * (Wb * Lb / 5 + Wa * Lb / 20 + La * Wb / 20 + Wa * La * (1 / 30)) * H ** 3
    elif La == Lb:
        L = La
        x2 = (1 / 24) * p * L ** 3 * H * (Wb + Wa)
        y2 = (1 / 48) * p * L * H * (Wb ** 3 + Wa * Wb ** 2 + Wa ** 2 * Wb + Wa ** 3)
        z2 = (1 / 12) * p * L * H ** 3 * (3 * Wb + Wa)
    else:
        W = Wa
        x2 = (1 / 48) * p * W * H * (Lb ** 3 + La * Lb ** 2 + La ** 2 * Lb + La ** 3)
        y2 = (1 / 24) * p * W ** 3 * H * (Lb + La)
        z2 = (1 / 12) * p * W * H ** 3 * (3 * Lb + La)
    return y2 + z2, x2 + z2, x2 + y2


def _place(M_local, mass, I_diag, R, center, integer=False):
    """6x6 mass matrix of a body with mass `mass` and principal MoI I_diag (member axes)
    about its CG, rotated to global axes (R^T I R with T = R^T, raft/raft_member.py:538-547)
    and translated to the PRP (translateMatrix6to6DOF with r = center).
    integer=True reproduces the reference's zero-length sections, whose `mass = 0` is a
    Python int: np.diag then builds an integer matrix and the assigned MoI block is
    truncated toward zero."""
    Mmat = np.diag([mass, mass, mass, 0.0, 0.0, 0.0])
    T = R.T
    Irot = T.T @ (np.diag(I_diag) @ T)
    Mmat[3:, 3:] = np.trunc(Irot) if integer else Irot
    return M_local + translate_matrix_6to6(Mmat, center)


# ------------------------------------------------------------------------ member inertia
def member_inertia(mem, rPRP=np.zeros(3)):
    """Mass, CG (relative to the PRP), shell mass, ballast masses and densities of one
    member; sets mem.M_struc, mem.vfill, mem.m_cap_list (raft/raft_member.py:307-707)."""
    mem.M_struc = np.zeros([6, 6])
    mem.vfill = []
    mass_center = np.zeros(3)
    mshell = 0.0
    mfill, pfill = [], []
    circ = mem.shape == "circular"
    Ixx = Iyy = Izz = 0.0
    for i in range(1, len(mem.stations)):
        l = mem.stations[i] - mem.stations[i - 1]
        if l == 0.0:
            # A zero-length section adds no mass, but the reference leaves the previous
            # section's principal moments in place and adds them again at the PRP
            # (raft/raft_member.py:420-426 set only mass/center/fill; :540-547 then use
            # Ixx/Iyy/Izz as left by the last section).  Kept for parity.
            mass, center, m_shell, v_fill, m_fill, rho_fill = 0.0, np.zeros(3), 0.0, 0.0, 0.0, 0.0
        else:
            rho_shell = mem.rho_shell
            l_fill = mem.l_fill if np.isscalar(mem.l_fill) else mem.l_fill[i - 1]
            rho_fill = mem.rho_fill if np.isscalar(mem.rho_fill) else mem.rho_fill[i - 1]
            if circ:
                dA, dB = mem.d[i - 1], mem.d[i]
                dAi, dBi = dA - 2 * mem.t[i - 1], dB - 2 * mem.t[i]
            else:
                dA, dB = mem.sl[i - 1], mem.sl[i]
                dAi, dBi = dA - 2 * mem.t[i - 1], dB - 2 * mem.t[i]
            V_o, hco = frustum_vcv(dA, dB, l)
            V_i, hci = frustum_vcv(dAi, dBi, l)
            v_shell = V_o - V_i
            m_shell = v_shell * rho_shell
            hc_shell = (hco * V_o - hci * V_i) / (V_o - V_i)
            dBi_fill = (dBi - dAi) * (l_fill / l) + dAi        # inner size at the ballast level
            v_fill, hc_fill = frustum_vcv(dAi, dBi_fill, l_fill)
            m_fill = v_fill * rho_fill
            mass = m_shell + m_fill
            hc = (hc_fill * m_fill + hc_shell * m_shell) / mass
            if circ:
                Ir_o, Ia_o = _frustum_moi(dA, dB, l, rho_shell)
                Ir_i, Ia_i = _frustum_moi(dAi, dBi, l, rho_shell)
                Ir_f, Ia_f = _frustum_moi(dAi, dBi_fill, l_fill, rho_fill)
                I_rad = (Ir_o - Ir_i) + Ir_f - mass * hc ** 2       # parallel axis to the CG
                Ixx = Iyy = I_rad
                Izz = (Ia_o - Ia_i) + Ia_f
            else:
                xo, yo, zo = _rect_frustum_moi(dA[0], dA[1], dB[0], dB[1], l, rho_shell)
                xi, yi, zi = _rect_frustum_moi(dAi[0], dAi[1], dBi[0], dBi[1], l, rho_shell)
                xf, yf, zf = _rect_frustum_moi(dAi[0], dAi[1], dBi_fill[0], dBi_fill[1], l_fill, rho_fill)
                Ixx = (xo - xi) + xf - mass * hc ** 2
                Iyy = (yo - yi) + yf - mass * hc ** 2
                Izz = (zo - zi) + zf
            center = mem.rA + mem.q * (mem.stations[i - 1] + hc) - rPRP
        mass_center = mass_center + mass * center
        mshell += m_shell
        mem.vfill.append(v_fill)
        mfill.append(m_fill)
        pfill.append(rho_fill)
        mem.M_struc = _place(mem.M_struc, mass, [Ixx, Iyy, Izz], mem.R, center, integer=(l == 0.0))

    # end caps and bulkheads (raft/raft_member.py:553-700), same material as the shell
    mem.m_cap_list = []
    for i in range(len(mem.cap_stations)):
        L, h = mem.cap_stations[i], mem.cap_t[i]
        rho_cap = mem.rho_shell
        st = mem.stations
        if circ:
            hole = mem.cap_d_in[i]
            dd = mem.d - 2 * mem.t
            dA, dB, dAi, dBi = _cap_sizes(L, h, i, st, dd, hole, mem.cap_stations, lambda x: np.interp(x, st, dd))
            V_o, hco = frustum_vcv(dA, dB, h)
            V_i, hci = frustum_vcv(dAi, dBi, h)
            m_cap = (V_o - V_i) * rho_cap
            hc_cap = (hco * V_o - hci * V_i) / (V_o - V_i)
            Ir_o, Ia_o = _frustum_moi(dA, dB, h, rho_cap)
            Ir_i, Ia_i = _frustum_moi(dAi, dBi, h, rho_cap)
            Ixx = Iyy = (Ir_o - Ir_i) - m_cap * hc_cap ** 2
            Izz = Ia_o - Ia_i
        else:
            # The reference's rectangular cap branch calls RectangularFrustumMOI with four
            # arguments (raft/raft_member.py:664-665) and so raises TypeError for any
            # rectangular member with caps; the same inputs fail here the same way.
            raise TypeError("RectangularFrustumMOI() missing 2 required positional arguments: 'H' and 'p'")
        pos = mem.rA + mem.q * L - rPRP
        if L == st[0]:
            center_cap = pos + mem.q * hc_cap
        elif L == st[-1]:
            center_cap = pos - mem.q * (h - hc_cap)
        else:
            center_cap = pos - mem.q * ((h / 2) - hc_cap)
        mass_center = mass_center + m_cap * center_cap
        mshell += m_cap
        mem.m_cap_list.append(m_cap)
        mem.M_struc = _place(mem.M_struc, m_cap, [Ixx, Iyy, Izz], mem.R, center_cap)

    mass = mem.M_struc[0, 0]
    return mass, mass_center / mass, mshell, mfill, pfill


def _cap_sizes(L, h, i, st, d, hole, cap_st, interp):
    """Outer/inner diameters at both faces of a circular cap or bulkhead of thickness h at
    station L (raft/raft_member.py:567-598)."""
    if L == st[0]:                    # bottom end cap
        dA, dB = d[0], interp(L + h)
        dAi = hole
        return dA, dB, dAi, dB * (dAi / dA)
    if L == st[-1]:                   # top end cap
        dA, dB = interp(L - h), d[-1]
        dBi = hole
        return dA, dB, dA * (dBi / dB), dBi
    if (st[0] < L < st[0] + h) or (st[-1] - h < L < st[-1]):
        raise ValueError("This setup cannot be handled by getIneria yet")
    if i < len(cap_st) - 1 and L == cap_st[i + 1]:     # discontinuity: cap below it
        dA, dB = interp(L - h), d[i]
        dBi = hole
        return dA, dB, dA * (dBi / dB), dBi
    if i > 0 and L == cap_st[i - 1]:                   # ... and the cap above it
        dA, dB = d[i], interp(L + h)
        dAi = hole
        return dA, dB, dAi, dB * (dAi / dA)
    dA, dB, dM = interp(L - h / 2), interp(L + h / 2), interp(L)   # mid-member bulkhead
    return dA, dB, dA * (hole / dM), dB * (hole / dM)


# ------------------------------------------------------------------- member hydrostatics
def _lin(x, xA, xB, yA, yB):
    """raft/helpers.py:341-343"""
    return yA + (x - xA) * (yB - yA) / (xB - xA)


def member_hydrostatics(mem, rPRP=np.zeros(3), rho=1025, g=9.81):
    """Buoyancy vector, hydrostatic stiffness, submerged volume, centre of buoyancy and
    waterplane properties of one member about the PRP (raft/raft_member.py:712-874)."""
    Fvec = np.zeros(6)
    Cmat = np.zeros([6, 6])
    V_UW = 0.0
    rV = np.zeros(3)
    AWP = IWP = xWP = yWP = 0.0
    circ = mem.shape == "circular"
    rHS = np.array([rPRP[0], rPRP[1], 0.0])
    for i in range(1, len(mem.stations)):
        rA = mem.rA + mem.q * mem.stations[i - 1] - rHS
        rB = mem.rA + mem.q * mem.stations[i] - rHS
        if rA[2] * rB[2] <= 0:        # segment crosses (or touches) the waterplane
            beta = np.arctan2(mem.q[1], mem.q[0])
            phi = np.arctan2(np.sqrt(mem.q[0] ** 2 + mem.q[1] ** 2), mem.q[2])
            cphi, sphi, tphi = np.cos(phi), np.sin(phi), np.tan(phi)
            cb, sb = np.cos(beta), np.sin(beta)
            xWP = _lin(0, rA[2], rB[2], rA[0], rB[0])
            yWP = _lin(0, rA[2], rB[2], rA[1], rB[1])
            if circ:
                dWP = _lin(0, rA[2], rB[2], mem.d[i], mem.d[i - 1])     # end values in the reference's order
                AWP = (np.pi / 4) * dWP ** 2
                IWP = (np.pi / 64) * dWP ** 4
                IxWP = IyWP = IWP
            else:
                slWP = _lin(0, rA[2], rB[2], mem.sl[i], mem.sl[i - 1])
                AWP = slWP[0] * slWP[1]
                Iloc = np.diag([(1 / 12) * slWP[0] * slWP[1] ** 3, (1 / 12) * slWP[0] ** 3 * slWP[1], 0.0])
                T = mem.R.T
                Irot = T.T @ Iloc @ T
                IxWP, IyWP = Irot[0, 0], Irot[1, 1]
            LWP = abs(rA[2] / cphi)
            V_i, hc = frustum_vcv(mem.d[i - 1], dWP, LWP) if circ else frustum_vcv(mem.sl[i - 1], slWP, LWP)
            rc = rA + mem.q * hc
            Fz = rho * g * V_i
            M = -rho * g * np.pi * (dWP ** 2 / 32 * (2.0 + tphi ** 2) + 0.5 * (rA[2] / cphi) ** 2) * sphi if circ else 0
            Fvec[2] += Fz
            Fvec[3] += M * (-sb) + Fz * rA[1]
            Fvec[4] += M * cb - Fz * rA[0]
            rg = rho * g
            Cmat[2, 2] += rg * AWP / cphi
            Cmat[2, 3] += rg * (-AWP * yWP)
            Cmat[2, 4] += rg * (AWP * xWP)
            Cmat[3, 2] += rg * (-AWP * yWP)
            Cmat[3, 3] += rg * (IxWP + AWP * yWP ** 2)
            Cmat[3, 4] += rg * (AWP * xWP * yWP)
            Cmat[4, 2] += rg * (AWP * xWP)
            Cmat[4, 3] += rg * (AWP * xWP * yWP)
            Cmat[4, 4] += rg * (IyWP + AWP * xWP ** 2)
            Cmat[3, 3] += rg * V_i * rc[2]
            Cmat[4, 4] += rg * V_i * rc[2]
            V_UW += V_i
            rV += rc * V_i
        elif rA[2] <= 0 and rB[2] <= 0:      # fully submerged segment
            lseg = mem.stations[i] - mem.stations[i - 1]
            V_i, hc = frustum_vcv(mem.d[i - 1], mem.d[i], lseg) if circ else frustum_vcv(mem.sl[i - 1], mem.sl[i], lseg)
            rc = rA + mem.q * hc
            f = np.array([0.0, 0.0, rho * g * V_i])
            Fvec[:3] += f
            Fvec[3:] += np.cross(rc, f)
            Cmat[3, 3] += rho * g * V_i * rc[2]
            Cmat[4, 4] += rho * g * V_i * rc[2]
            V_UW += V_i
            rV += rc * V_i
    mem.V = V_UW
    r_center = rV / V_UW if V_UW > 0 else np.zeros(3)
    return Fvec, Cmat, V_UW, r_center, AWP, IWP, xWP, yWP


# --------------------------------------------------------------------------- RNA (rotor)
class RNA:
    """Rotor-nacelle assembly inertia and pose: the parts of raft/raft_rotor.py:42-111 and
    376-458 that calcStatics reads (no aerodynamics)."""

    def __init__(self, turbine, ir, get):
        nr = turbine["nrotors"]
        if "rRNA" in turbine:
            self.r_rel = np.array(get(turbine, "rRNA", shape=[nr, 3])[ir], dtype=float)
        else:
            if nr > 1:
                raise Exception("For designs with more than one rotor, the RNA reference point must be specified "
                                "for each of them.")
            self.r_rel = np.array([0, 0, 100.0])
        self.overhang = get(turbine, "overhang", shape=nr)[ir]
        self.xCG_RNA = get(turbine, "xCG_RNA", shape=nr)[ir]
        self.mRNA = get(turbine, "mRNA", shape=nr)[ir]
        self.IxRNA = get(turbine, "IxRNA", shape=nr)[ir]
        self.IrRNA = get(turbine, "IrRNA", shape=nr)[ir]
        self.shaft_tilt = get(turbine, "shaft_tilt", shape=nr)[ir] * np.pi / 180
        self.shaft_toe = get(turbine, "shaft_toe", shape=nr, default=0)[ir] * np.pi / 180
        self.yaw_mode = int(get(turbine, "yaw_mode", shape=nr, dtype=int, default=0)[ir])
        self.yaw_command = 0.0
        self.inflow_heading = 0.0
        self.turbine_heading = 0.0
        self.yaw = 0.0
        q = rotation_matrix(0, self.shaft_tilt, self.shaft_toe) @ np.array([1.0, 0.0, 0.0])
        if "hHub" in turbine:
            self.r_rel[2] = get(turbine, "hHub", shape=nr)[ir] - q[2] * self.overhang
        self.setPosition(np.zeros(6))

    def setPosition(self, r6):
        """raft/raft_rotor.py:376-409 with setYaw (:412-458)"""
        R_ptfm = rotation_matrix(*r6[3:])
        heading = r6[5]
        if self.yaw_mode == 0:
            self.yaw = self.inflow_heading - heading + self.yaw_command
        elif self.yaw_mode == 1:
            self.yaw = self.turbine_heading - heading
        elif self.yaw_mode == 2:
            self.yaw = self.yaw_command
        elif self.yaw_mode == 3:
            self.yaw = self.yaw_command - heading
        else:
            raise Exception("Unsupported yaw_mode value. Must be 0, 1, or 2.")
        self.turbine_heading = heading + self.yaw
        R_q_rel = rotation_matrix(0, self.shaft_tilt, self.shaft_toe + self.yaw)
        self.R_q = R_q_rel @ R_ptfm
        self.q = R_ptfm @ (R_q_rel @ np.array([1.0, 0.0, 0.0]))
        self.r_RRP_rel = R_ptfm @ self.r_rel
        self.r_CG_rel = self.r_RRP_rel + self.q * self.xCG_RNA
        self.r_hub_rel = self.r_RRP_rel + self.q * self.overhang
        self.r3 = np.asarray(r6[:3]) + self.r_hub_rel


def _rotate3(M, R):
    """rotateMatrix3: R M R^T (raft/helpers.py)"""
    return R @ M @ R.T


def _rotate6(M, R):
    """rotateMatrix6 of a 2-D 6x6 tensor (raft/helpers.py:507-531)"""
    out = np.zeros_like(M)
    out[:3, :3] = _rotate3(M[:3, :3], R)
    out[:3, 3:] = _rotate3(M[:3, 3:], R)
    out[3:, :3] = out[:3, 3:].T
    out[3:, 3:] = _rotate3(M[3:, 3:], R)
    return out


# ------------------------------------------------------------------------- FOWT totals
def fowt_statics(fowt):
    """FOWT.calcStatics (raft/raft_fowt.py:291-565) for members and RNAs above water:
    sets M_struc, B_struc, C_struc, W_struc, C_hydro, W_hydro and the derived properties
    (rCG, rCG_sub, m_ballast, rCB, m, V, AWP, rM, props, ...) on `fowt`."""
    rho, g = fowt.rho_water, fowt.g
    r6 = fowt.r6
    fowt.M_struc = np.zeros([6, 6])
    fowt.B_struc = np.zeros([6, 6])
    fowt.C_struc = np.zeros([6, 6])
    fowt.W_struc = np.zeros(6)
    fowt.C_hydro = np.zeros([6, 6])
    fowt.W_hydro = np.zeros(6)
    VTOT = AWP_TOT = IWPx_TOT = IWPy_TOT = 0.0
    Sum_V_rCB = np.zeros(3)
    Sum_AWP_rWP = np.zeros(2)
    m_center_sum = np.zeros(3)
    fowt.m_sub = 0.0
    fowt.C_struc_sub = np.zeros([6, 6])
    fowt.M_struc_sub = np.zeros([6, 6])
    m_sub_sum = np.zeros(3)
    fowt.m_shell = 0.0
    mballast, pballast = [], []
    fowt.mtower = np.zeros(fowt.ntowers)
    fowt.rCG_tow = []

    def add_hydro(mem):
        nonlocal VTOT, AWP_TOT, IWPx_TOT, IWPy_TOT, Sum_V_rCB, Sum_AWP_rWP
        Fvec, Cmat, V_UW, r_CB, AWP, IWP, xWP, yWP = member_hydrostatics(mem, rPRP=r6[:3], rho=rho, g=g)
        fowt.W_hydro += Fvec
        fowt.C_hydro += Cmat
        VTOT += V_UW
        AWP_TOT += AWP
        IWPx_TOT += IWP + AWP * yWP ** 2
        IWPy_TOT += IWP + AWP * xWP ** 2
        Sum_V_rCB = Sum_V_rCB + r_CB * V_UW
        Sum_AWP_rWP = Sum_AWP_rWP + np.array([xWP, yWP]) * AWP

    mems = [m for m in fowt.memberList if m.name != "nacelle"]
    for i, mem in enumerate(mems):
        mem.setPosition(r6=r6)
        mass, center, m_shell, mfill, pfill = member_inertia(mem, rPRP=r6[:3])
        fowt.W_struc[:3] += np.array([0.0, 0.0, -g * mass])
        fowt.W_struc[3:] += np.cross(center, np.array([0.0, 0.0, -g * mass]))
        fowt.M_struc += mem.M_struc
        m_center_sum = m_center_sum + center * mass
        if mem.type <= 1:                      # tower (raft/raft_fowt.py:356-358)
            fowt.mtower[i - fowt.nplatmems] = mass
            fowt.rCG_tow.append(center)
        if mem.type > 1:                       # substructure
            fowt.m_sub += mass
            fowt.M_struc_sub += mem.M_struc
            m_sub_sum = m_sub_sum + center * mass
            fowt.m_shell += m_shell
            mballast.extend(mfill)
            pballast.extend(pfill)
        add_hydro(mem)
    for mem in (m for m in fowt.memberList if m.name == "nacelle"):
        add_hydro(mem)                          # buoyancy only (:447-464)
    for rot in fowt.rnaList:
        Mmat = _rotate6(np.diag([rot.mRNA, rot.mRNA, rot.mRNA, rot.IxRNA, rot.IrRNA, rot.IrRNA]), rot.R_q)
        f = np.array([0.0, 0.0, -g * rot.mRNA])
        fowt.W_struc[:3] += f
        fowt.W_struc[3:] += np.cross(rot.r_CG_rel, f)
        fowt.M_struc += translate_matrix_6to6(Mmat, rot.r_CG_rel)
        m_center_sum = m_center_sum + rot.r_CG_rel * rot.mRNA

    m_all = fowt.M_struc[0, 0]
    rCG_all = m_center_sum / m_all
    fowt.rCG = rCG_all
    fowt.rCG_sub = m_sub_sum / fowt.m_sub
    M_sub = translate_matrix_6to6(fowt.M_struc_sub, -fowt.rCG_sub)
    M_all = translate_matrix_6to6(fowt.M_struc, -fowt.rCG)
    fowt.pb = []
    for p in pballast:                         # unique nonzero ballast densities, first-seen order
        if p != 0 and fowt.pb.count(p) == 0:
            fowt.pb.append(p)
    fowt.m_ballast = np.zeros(len(fowt.pb))
    for i, p in enumerate(fowt.pb):
        for m, pp in zip(mballast, pballast):
            if float(pp) == float(p):
                fowt.m_ballast[i] += m
    rCB_TOT = Sum_V_rCB / VTOT
    zMeta = 0 if VTOT == 0 else rCB_TOT[2] + IWPx_TOT / VTOT
    fowt.C_struc[3, 3] = fowt.C_struc[4, 4] = -m_all * g * rCG_all[2]
    fowt.C_struc_sub[3, 3] = fowt.C_struc_sub[4, 4] = -fowt.m_sub * g * fowt.rCG_sub[2]
    fowt.rCB = rCB_TOT
    fowt.m = m_all
    fowt.V = VTOT
    fowt.AWP = AWP_TOT
    fowt.rM = np.array([rCB_TOT[0], rCB_TOT[1], zMeta])
    fowt.props = {"m": fowt.m, "m_sub": fowt.m_sub, "v": fowt.V, "rCG": fowt.rCG, "rCG_sub": fowt.rCG_sub,
                  "rCB": fowt.rCB, "AWP": fowt.AWP, "rM": fowt.rM, "Ixx": M_all[3, 3], "Iyy": M_all[4, 4],
                  "Izz": M_all[5, 5], "Ixx_sub": M_sub[3, 3], "Iyy_sub": M_sub[4, 4], "Izz_sub": M_sub[5, 5]}
