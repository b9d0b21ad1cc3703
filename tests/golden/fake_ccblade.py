"""A scripted stand-in for CCBlade (test infrastructure only).

CCBlade (WISDEM) is a third-party dependency of the reference's rotor path
(raft/raft_rotor.py:17-20) and is not installed here.  To pin RAFT's OWN rotor code -- the
CCBlade inputs it builds (polars, blade tables) and the aero-servo linearisation it derives
from CCBlade's loads and derivatives (Rotor.calcAero, raft/raft_rotor.py:788-1005) -- both the
reference (tests/golden/make_golden.py golden_rotor) and this build (tests/test_rotor.py) are
run with this same object: it records every constructor argument and returns loads and
derivatives that are fixed smooth functions of (Uinf, Omega, pitch, tilt, yaw).  The values
mean nothing physically; they only have to be identical on both sides.
"""
import numpy as np


class FakeAirfoil:
    def __init__(self, alpha, Re, cl, cd, cm):
        self.alpha, self.Re = np.asarray(alpha, dtype=float), Re
        self.cl, self.cd, self.cm = (np.asarray(x, dtype=float) for x in (cl, cd, cm))


class FakeCCBlade:
    def __init__(self, r, chord, theta, af, Rhub, Rtip, B, rho, mu, precone, tilt, yaw, shearExp, hubHt, nSector,
                 precurve, precurveTip, presweep, presweepTip, **flags):
        self.args = dict(r=np.asarray(r, dtype=float), chord=np.asarray(chord, dtype=float),
                         theta=np.asarray(theta, dtype=float), Rhub=float(Rhub), Rtip=float(Rtip), B=float(B),
                         rho=float(rho), mu=float(mu), precone=float(precone), tilt=float(tilt), yaw=float(yaw),
                         shearExp=float(shearExp), hubHt=float(hubHt), nSector=float(nSector),
                         precurve=np.asarray(precurve, dtype=float), precurveTip=float(precurveTip),
                         presweep=np.asarray(presweep, dtype=float), presweepTip=float(presweepTip),
                         cl=np.array([a.cl for a in af]), cd=np.array([a.cd for a in af]),
                         cm=np.array([a.cm for a in af]), alpha=af[0].alpha)
        self.flags = flags
        self.tilt = np.radians(tilt)
        self.yaw = np.radians(yaw)
        self.calls = []

    def evaluate(self, Uinf, Omega_rpm, pitch_deg, coefficients=False):
        U = float(np.atleast_1d(Uinf)[0])
        Om = float(np.atleast_1d(Omega_rpm)[0])
        pi = float(np.atleast_1d(pitch_deg)[0])
        c = np.cos(self.tilt) * np.cos(self.yaw)
        s = np.sin(self.yaw) + 0.3 * np.sin(self.tilt)
        self.calls.append((U, Om, pi, float(self.tilt), float(self.yaw)))
        T = 1.1e4 * U * U * c / (1.0 + 0.02 * pi * pi) + 3e3 * Om
        Q = 2.3e5 * U * (1 + 0.01 * Om) * c / (1.0 + 0.05 * pi)
        loads = {"T": np.array([T]), "Q": np.array([Q]), "P": np.array([Q * Om * np.pi / 30]),
                 "Y": np.array([1.7e3 * U * s]), "Z": np.array([-9e2 * U * s]), "My": np.array([4.1e4 * U * s]),
                 "Mz": np.array([-2.2e4 * U * c + 5e3 * s]), "Mb": np.array([T * 31.0]), "CP": np.array([0.45]),
                 "CT": np.array([0.8]), "CQ": np.array([0.05]), "CY": np.array([0.0]), "CZ": np.array([0.0]),
                 "CMy": np.array([0.0]), "CMz": np.array([0.0]), "CMb": np.array([0.1])}
        dT = {"dUinf": np.array([[2.2e4 * U * c / (1.0 + 0.02 * pi * pi) + 150.0 * Om]]),
              "dOmega": np.array([[3e3 + 41.0 * U]]),
              "dpitch": np.array([[-1.1e4 * U * U * c * 0.04 * pi / (1.0 + 0.02 * pi * pi) ** 2 - 7e3 * U]])}
        dQ = {"dUinf": np.array([[2.3e5 * (1 + 0.01 * Om) * c / (1.0 + 0.05 * pi)]]),
              "dOmega": np.array([[2.3e3 * U * c / (1.0 + 0.05 * pi) - 1.5e5]]),
              "dpitch": np.array([[-2.3e5 * U * (1 + 0.01 * Om) * c * 0.05 / (1.0 + 0.05 * pi) ** 2 - 2e4 * U]])}
        derivs = {"dT": dT, "dQ": dQ, "dP": {"dr": np.zeros((1, len(self.args["r"])))}}
        return loads, derivs
