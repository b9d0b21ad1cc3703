"""Blade-element momentum rotor loads: a restatement of CCBlade, the third-party BEM solver the
reference's rotor layer calls (raft/raft_rotor.py:17-20, :331-370, :699-768; WISDEM/CCBlade,
absent from this image).

This is the published method of S. Andrew Ning, "A simple solution method for the blade
element momentum equations with guaranteed convergence", Wind Energy 17 (2014), as CCBlade
implements it:
  * the residual is a function of the inflow angle phi alone,
        phi > 0:  f(phi) = sin(phi) / (1 - a) - cos(phi) / lambda_r * (1 - kp)
        phi < 0:  f(phi) = sin(phi) (1 - k) - cos(phi) / lambda_r * (1 - kp)
    with k = sigma' cn / (4 F sin^2 phi), kp = sigma' ct / (4 F sin phi cos phi),
    sigma' = B c / (2 pi r), F = Ftip Fhub (Prandtl), a = k / (1 + k) in the momentum region
    and Buhl's empirical correction past k = 2/3, ap = kp / (1 - kp);
  * its root is bracketed in (0, pi/2] (else [-pi/4, 0) or [pi/2, pi)) and found with Brent's
    method; alpha = phi - (theta + pitch), cl and cd from the airfoil's smoothing splines;
  * the section loads Np = cn q c, Tp = ct q c use the converged inductions
    (W = |(Vx (1 - a), Vy (1 + ap))|);
  * inflow per section and azimuth from the hub wind speed (power-law shear over the height
    above the hub), rotor tilt and yaw, and the rotation; blade precone / precurve / presweep
    through the azimuthal coordinates;
  * thrust and torque by trapezoidal integration along the blade path with zero loads at the
    hub and tip radii, averaged over nSector azimuthal sectors (1 sector when tilt, yaw and
    shear are all zero).
Derivatives with respect to Uinf, Omega and pitch (what RAFT consumes, raft/raft_rotor.py:
826-832) follow the solution through the residual: dphi/dx = -(df/dx) / (df/dphi) per section,
the partial derivatives by central differences of the closed-form residual and load functions
at the converged phi (no re-solve).

Parity: pinned only through the reference's own literal expectations that depend on rotor
thrust (tests/test_model.py desired_X0 'wind' / 'wind_wave_current' and desired_fn 'loaded',
tests/test_ccblade.py).  Beyond those values CCBlade's arithmetic is "parity unpinned".
"""
import numpy as np
from scipy.interpolate import RectBivariateSpline
from scipy.optimize import brentq


class CCAirfoil:
    """Airfoil polars as smoothing bicubic splines over (alpha, Re).  One Reynolds number (the
    reference passes none, raft/raft_rotor.py:334) is widened to two identical columns, so the
    polars are Re-independent."""

    def __init__(self, alpha, Re, cl, cd, cm=(), x=(), y=(), AFName="DEFAULTAF"):
        alpha = np.deg2rad(np.asarray(alpha, dtype=float))
        Re = list(np.atleast_1d(Re)) if np.size(Re) else []
        cl = np.asarray(cl, dtype=float)
        cd = np.asarray(cd, dtype=float)
        cm = np.asarray(cm, dtype=float) if np.size(cm) else np.zeros(0)
        self.use_cm = cm.size > 0
        self.one_Re = False
        if len(Re) < 2:
            Re = [1e1, 1e15]
            cl = np.c_[cl, cl]
            cd = np.c_[cd, cd]
            if self.use_cm:
                cm = np.c_[cm, cm]
            self.one_Re = True
        kx = min(len(alpha) - 1, 3)
        ky = min(len(Re) - 1, 3)
        # a small amount of smoothing is used to prevent spurious multiple solutions
        self.cl_spline = RectBivariateSpline(alpha, Re, cl, kx=kx, ky=ky, s=0.1)
        self.cd_spline = RectBivariateSpline(alpha, Re, cd, kx=kx, ky=ky, s=0.001)
        if self.use_cm:
            self.cm_spline = RectBivariateSpline(alpha, Re, cm, kx=kx, ky=ky, s=0.0001)
        self.alpha = alpha

    def evaluate(self, alpha, Re, return_cm=False):
        cl = self.cl_spline.ev(alpha, Re)
        cd = self.cd_spline.ev(alpha, Re)
        if return_cm:
            return cl, cd, (self.cm_spline.ev(alpha, Re) if self.use_cm else 0.0 * cl)
        return cl, cd


def define_curvature(r, precurve, presweep, precone):
    """Azimuthal coordinates of the blade stations, local cone angle, path length."""
    x_az = -r * np.sin(precone) + precurve * np.cos(precone)
    z_az = r * np.cos(precone) + precurve * np.sin(precone)
    y_az = presweep
    n = len(r)
    cone = np.zeros(n)
    seg = np.arctan2(-(x_az[1:] - x_az[:-1]), z_az[1:] - z_az[:-1])
    cone[0] = seg[0]
    cone[1:-1] = 0.5 * (seg[:-1] + seg[1:])
    cone[-1] = seg[-1]
    s = np.zeros(n)
    s[1:] = np.cumsum(np.sqrt((precurve[1:] - precurve[:-1]) ** 2 + (presweep[1:] - presweep[:-1]) ** 2 +
                              (r[1:] - r[:-1]) ** 2))
    return x_az, y_az, z_az, cone, s


def wind_components(r, precurve, presweep, precone, yaw, tilt, azimuth, Uinf, OmegaRPM, hubHt, shearExp):
    """Axial (Vx) and tangential (Vy) inflow of each section at one azimuth (radians)."""
    sy, cy = np.sin(yaw), np.cos(yaw)
    st, ct = np.sin(tilt), np.cos(tilt)
    sa, ca = np.sin(azimuth), np.cos(azimuth)
    Omega = OmegaRPM * np.pi / 30.0
    x_az, y_az, z_az, cone, s = define_curvature(r, precurve, presweep, precone)
    sc, cc = np.sin(cone), np.cos(cone)
    heightFromHub = (y_az * sa + z_az * ca) * ct - x_az * st
    V = Uinf * (1.0 + heightFromHub / hubHt) ** shearExp
    Vwind_x = V * ((cy * st * ca + sy * sa) * sc + cy * ct * cc)
    Vwind_y = V * (cy * st * sa - sy * ca)
    Vrot_x = -Omega * y_az * sc
    Vrot_y = Omega * z_az
    return Vwind_x + Vrot_x, Vwind_y + Vrot_y


def relative_wind(phi, a, ap, Vx, Vy, pitch, chord, theta, rho, mu):
    if abs(a) > 10:
        W = Vy * (1 + ap) / np.cos(phi)
    elif abs(ap) > 10:
        W = Vx * (1 - a) / np.sin(phi)
    else:
        W = np.sqrt((Vx * (1 - a)) ** 2 + (Vy * (1 + ap)) ** 2)
    return phi - (theta + pitch), W, rho * W * chord / mu


def induction_factors(r, chord, Rhub, Rtip, phi, cl, cd, B, Vx, Vy, usecd, hubloss, tiploss, wakerotation):
    """The BEM residual and the induction factors at inflow angle phi (Ning 2014, eqs. 5-20)."""
    sigma_p = B / 2.0 / np.pi * chord / r
    sphi, cphi = np.sin(phi), np.cos(phi)
    if usecd:
        cn = cl * cphi + cd * sphi
        ct = cl * sphi - cd * cphi
    else:
        cn = cl * cphi
        ct = cl * sphi
    Ftip = 1.0
    if tiploss:
        factortip = B / 2.0 * (Rtip - r) / (r * abs(sphi))
        Ftip = 2.0 / np.pi * np.arccos(np.exp(-factortip))
    Fhub = 1.0
    if hubloss:
        factorhub = B / 2.0 * (r - Rhub) / (Rhub * abs(sphi))
        Fhub = 2.0 / np.pi * np.arccos(np.exp(-factorhub))
    F = Ftip * Fhub
    k = sigma_p * cn / 4.0 / F / sphi / sphi
    kp = sigma_p * ct / 4.0 / F / sphi / cphi
    if phi > 0:   # momentum / empirical region
        if k <= 2.0 / 3.0:
            a = k / (1 + k)
        else:   # Glauert correction (Buhl)
            g1 = 2.0 * F * k - (10.0 / 9 - F)
            g2 = 2.0 * F * k - (4.0 / 3 - F) * F
            g3 = 2.0 * F * k - (25.0 / 9 - 2 * F)
            if abs(g3) < 1e-6:
                a = 1.0 - 1.0 / 2.0 / np.sqrt(g2)
            else:
                a = (g1 - np.sqrt(g2)) / g3
    else:         # propeller brake region
        a = k / (k - 1.0) if k > 1.0 else 0.0
    ap = kp / (1.0 - kp)
    if not wakerotation:
        ap = 0.0
        kp = 0.0
    lambda_r = Vy / Vx
    if phi > 0:
        fzero = sphi / (1.0 - a) - cphi / lambda_r * (1.0 - kp)
    else:
        fzero = sphi * (1.0 - k) - cphi / lambda_r * (1.0 - kp)
    return fzero, a, ap


def thrust_torque(Np, Tp, r, precurve, presweep, precone, Rhub, Rtip, precurveTip, presweepTip, azimuth=0.0):
    """One blade's hub loads at one azimuth [rad]: trapezoidal integration along the blade path,
    the section loads going to zero at the hub and tip radii.
      T  = int Np cos(cone) ds                           (shaft thrust)
      Q  = int Tp z_az ds                                (shaft torque)
      Y  = int [Tp cos(az) - Np sin(cone) sin(az)] ds    (in-plane side force, hub frame)
      Z  = int [Tp sin(az) + Np sin(cone) cos(az)] ds    (in-plane vertical force)
      My = cos(az) int Np z_az ds,  Mz = sin(az) int Np z_az ds   (the flapwise moment turned
                                                         into the hub frame by the azimuth)
    The side loads were identified against the reference's own expectations that depend on
    them (tests/test_model.py desired_X0 'wind': sway, heave, roll and yaw), see DESIGN.md §2."""
    rfull = np.r_[Rhub, r, Rtip]
    curvefull = np.r_[0.0, precurve, precurveTip]
    sweepfull = np.r_[0.0, presweep, presweepTip]
    Npfull = np.r_[0.0, Np, 0.0]
    Tpfull = np.r_[0.0, Tp, 0.0]
    x_az, y_az, z_az, cone, s = define_curvature(rfull, curvefull, sweepfull, precone)
    ds = s[1:] - s[:-1]

    def trap(g):
        return np.sum(ds * 0.5 * (g[:-1] + g[1:]))

    sa, ca = np.sin(azimuth), np.cos(azimuth)
    radial = Npfull * np.sin(cone)
    T = trap(Npfull * np.cos(cone))
    Q = trap(Tpfull * z_az)
    Y = trap(Tpfull * ca - radial * sa)
    Z = trap(Tpfull * sa + radial * ca)
    Mflap = trap(Npfull * z_az)
    return T, Q, Y, Z, Mflap * ca, Mflap * sa


class CCBlade:
    """The rotor: blade geometry, airfoils and operating environment (CCBlade's constructor
    signature, as raft/raft_rotor.py:338-370 calls it; angles in degrees on input)."""

    def __init__(self, r, chord, theta, af, Rhub, Rtip, B=3, rho=1.225, mu=1.81206e-5, precone=0.0, tilt=0.0,
                 yaw=0.0, shearExp=0.2, hubHt=80.0, nSector=8, precurve=None, precurveTip=0.0, presweep=None,
                 presweepTip=0.0, tiploss=True, hubloss=True, wakerotation=True, usecd=True, iterRe=1,
                 derivatives=False):
        self.r = np.array(r, dtype=float)
        self.chord = np.array(chord, dtype=float)
        self.theta = np.radians(np.array(theta, dtype=float))
        self.af = af
        self.Rhub, self.Rtip, self.B = float(Rhub), float(Rtip), int(B)
        self.rho, self.mu = float(rho), float(mu)
        self.precone = np.radians(precone)
        self.tilt = np.radians(tilt)
        self.yaw = np.radians(yaw)
        self.shearExp = float(shearExp)
        self.hubHt = float(hubHt)
        self.bemoptions = dict(usecd=usecd, tiploss=tiploss, hubloss=hubloss, wakerotation=wakerotation)
        self.iterRe = iterRe
        self.derivatives = derivatives
        n = len(self.r)
        self.precurve = np.zeros(n) if precurve is None else np.array(precurve, dtype=float)
        self.presweep = np.zeros(n) if presweep is None else np.array(presweep, dtype=float)
        self.precurveTip, self.presweepTip = float(precurveTip), float(presweepTip)
        self.rotorR = self.Rtip * np.cos(self.precone) + self.precurveTip * np.sin(self.precone)
        # azimuthal discretisation: one sector is enough for an axisymmetric inflow
        if self.tilt == 0.0 and self.yaw == 0.0 and self.shearExp == 0.0:
            self.nSector = 1
        else:
            self.nSector = max(4, int(nSector))

    # ------------------------------------------------------------------ one section
    def _run_bem(self, phi, r, chord, theta, af, Vx, Vy):
        a = ap = 0.0
        for _ in range(self.iterRe):
            alpha, W, Re = relative_wind(phi, a, ap, Vx, Vy, self.pitch, chord, theta, self.rho, self.mu)
            cl, cd = af.evaluate(alpha, Re)
            fzero, a, ap = induction_factors(r, chord, self.Rhub, self.Rtip, phi, cl, cd, self.B, Vx, Vy,
                                             **self.bemoptions)
        return fzero, a, ap

    def _errf(self, phi, *args):
        return self._run_bem(phi, *args)[0]

    def _loads(self, phi, rotating, r, chord, theta, af, Vx, Vy):
        cphi, sphi = np.cos(phi), np.sin(phi)
        if rotating:
            _, a, ap = self._run_bem(phi, r, chord, theta, af, Vx, Vy)
        else:
            a = ap = 0.0
        alpha, W, Re = relative_wind(phi, a, ap, Vx, Vy, self.pitch, chord, theta, self.rho, self.mu)
        cl, cd = af.evaluate(alpha, Re)
        cn = cl * cphi + cd * sphi   # these always contain drag
        ct = cl * sphi - cd * cphi
        q = 0.5 * self.rho * W ** 2
        return cn * q * chord, ct * q * chord, a, ap, alpha, cl, cd, W

    def _solve_phi(self, rotating, args):
        if not rotating:
            return np.pi / 2.0
        errf = self._errf
        eps = 1e-6
        lo, hi = eps, np.pi / 2
        if errf(lo, *args) * errf(hi, *args) > 0:   # an uncommon but possible case
            if errf(-np.pi / 4, *args) < 0 and errf(-eps, *args) > 0:
                lo, hi = -np.pi / 4, -eps
            else:
                lo, hi = np.pi / 2, np.pi - eps
        try:
            return brentq(errf, lo, hi, args=args)
        except ValueError:
            return 0.0

    def distributedAeroLoads(self, Uinf, Omega, pitch, azimuth):
        """Section loads Np, Tp [N/m] (and the BEM state) at one azimuth [deg]."""
        self.pitch = np.radians(pitch)
        Vx, Vy = wind_components(self.r, self.precurve, self.presweep, self.precone, self.yaw, self.tilt,
                                 np.radians(azimuth), Uinf, Omega, self.hubHt, self.shearExp)
        n = len(self.r)
        out = {k: np.zeros(n) for k in ("Np", "Tp", "a", "ap", "alpha", "Cl", "Cd", "W", "phi")}
        rotating = Omega != 0
        for i in range(n):
            args = (self.r[i], self.chord[i], self.theta[i], self.af[i], Vx[i], Vy[i])
            phi = self._solve_phi(rotating, args)
            Np, Tp, a, ap, alpha, cl, cd, W = self._loads(phi, rotating, *args)
            for k, v in zip(("Np", "Tp", "a", "ap", "alpha", "Cl", "Cd", "W", "phi"),
                            (Np, Tp, a, ap, alpha, cl, cd, W, phi)):
                out[k][i] = v
        self._Vx, self._Vy = Vx, Vy
        return out, {}

    # ------------------------------------------------------------------ section derivatives
    def _section_derivs(self, i, phi, Uinf, Omega, pitch, azimuth, rotating):
        """d(Np, Tp)/d(Uinf, Omega, pitch) of section i at the converged phi: partials of the
        residual and the load functions by central differences, dphi/dx = -f_x / f_phi."""
        r, chord, theta, af = self.r[i], self.chord[i], self.theta[i], self.af[i]

        def state(U, Om, pit):
            Vx, Vy = wind_components(self.r, self.precurve, self.presweep, self.precone, self.yaw, self.tilt,
                                     np.radians(azimuth), U, Om, self.hubHt, self.shearExp)
            return Vx[i], Vy[i], np.radians(pit)

        def f_and_loads(ph, U, Om, pit):
            Vx, Vy, self.pitch = state(U, Om, pit)
            args = (r, chord, theta, af, Vx, Vy)
            f = self._errf(ph, *args) if rotating else 0.0
            Np, Tp = self._loads(ph, rotating, *args)[:2]
            return np.array([f, Np, Tp])

        x0 = np.array([Uinf, Omega, pitch], dtype=float)
        hphi = 1e-7 * max(1.0, abs(phi))
        g_phi = (f_and_loads(phi + hphi, *x0) - f_and_loads(phi - hphi, *x0)) / (2 * hphi)
        dN, dT = np.zeros(3), np.zeros(3)
        for k in range(3):
            h = 1e-6 * max(1.0, abs(x0[k]))
            xp, xm = x0.copy(), x0.copy()
            xp[k] += h
            xm[k] -= h
            g_x = (f_and_loads(phi, *xp) - f_and_loads(phi, *xm)) / (2 * h)
            dphi = -g_x[0] / g_phi[0] if rotating and g_phi[0] != 0 else 0.0
            dN[k] = g_x[1] + g_phi[1] * dphi
            dT[k] = g_x[2] + g_phi[2] * dphi
        self.pitch = np.radians(pitch)
        return dN, dT

    # ------------------------------------------------------------------ rotor
    def evaluate(self, Uinf, Omega, pitch, coefficients=False):
        """Rotor loads (T, Y, Z, Q, My, Mz, P, Mb and, with coefficients, CT ... CMb) averaged over
        the azimuthal sectors, and their derivatives with respect to Uinf, Omega, pitch."""
        Uinf = np.atleast_1d(np.asarray(Uinf, dtype=float)).ravel()
        Omega = np.atleast_1d(np.asarray(Omega, dtype=float)).ravel()
        pitch = np.atleast_1d(np.asarray(pitch, dtype=float)).ravel()
        npts = len(Uinf)
        args = (self.r, self.precurve, self.presweep, self.precone, self.Rhub, self.Rtip, self.precurveTip,
                self.presweepTip)
        keys = ("T", "Y", "Z", "Q", "My", "Mz", "Mb")
        L = {k: np.zeros(npts) for k in keys}
        dTx = np.zeros((npts, 3))
        dQx = np.zeros((npts, 3))
        nsec = self.nSector
        for i in range(npts):
            for j in range(nsec):
                azimuth = 360.0 * float(j) / nsec
                loads, _ = self.distributedAeroLoads(Uinf[i], Omega[i], pitch[i], azimuth)
                sub = thrust_torque(loads["Np"], loads["Tp"], *args, azimuth=np.radians(azimuth))
                for k, v in zip(("T", "Q", "Y", "Z", "My", "Mz"), sub):
                    L[k][i] += self.B * v / nsec
                L["Mb"][i] += np.hypot(sub[4], sub[5]) / nsec   # one blade's flapwise root moment (unpinned)
                if self.derivatives:
                    rot = Omega[i] != 0
                    n = len(self.r)
                    dNp, dTp = np.zeros((n, 3)), np.zeros((n, 3))
                    for s_ in range(n):
                        dNp[s_], dTp[s_] = self._section_derivs(s_, loads["phi"][s_], Uinf[i], Omega[i], pitch[i],
                                                                azimuth, rot)
                    for k in range(3):   # T and Q are linear in the section loads
                        dt, dq = thrust_torque(dNp[:, k], dTp[:, k], *args)[:2]
                        dTx[i, k] += self.B * dt / nsec
                        dQx[i, k] += self.B * dq / nsec
            if nsec == 1:   # axisymmetric inflow: the B blades' in-plane loads cancel (unpinned case)
                for k in ("Y", "Z", "My", "Mz"):
                    L[k][i] = 0.0
        P = L["Q"] * Omega * np.pi / 30.0
        loads = dict(L, P=P)
        derivs = {}
        if self.derivatives:
            def block(d):
                return {"dUinf": np.diag(d[:, 0]), "dOmega": np.diag(d[:, 1]), "dpitch": np.diag(d[:, 2]),
                        "dr": np.zeros((npts, len(self.r)))}
            derivs["dT"] = block(dTx)
            derivs["dQ"] = block(dQx)
            derivs["dP"] = block(dQx * (Omega * np.pi / 30.0)[:, None] + np.c_[0 * Uinf, L["Q"] * np.pi / 30.0, 0 * Uinf])
        if coefficients:
            q = 0.5 * self.rho * Uinf ** 2
            A = np.pi * self.rotorR ** 2
            loads.update(CP=P / (q * A * Uinf), CT=L["T"] / (q * A), CY=L["Y"] / (q * A), CZ=L["Z"] / (q * A),
                         CQ=L["Q"] / (q * self.rotorR * A), CMy=L["My"] / (q * self.rotorR * A),
                         CMz=L["Mz"] / (q * self.rotorR * A), CMb=L["Mb"] / (q * self.rotorR * A))
        return loads, derivs
