"""Model: the frequency-domain response solve of a (multi-)FOWT system on MI355X.

Drop-in for the reference entry points on the hot path (raft/raft_model.py):
  Model(design)                   frequency grid + FOWTs                 :30-170
  Model.solveDynamics(case, ...)  drag fixed point + system response     :852-1146
  Model.analyzeCases(...)         per-case loop + motion outputs          :244-388
plus the batched form the reference does not have:
  Model.analyzeCasesBatch(cases)  every case in ONE device call (one workgroup per case).

Mean offsets (solveStatics: MoorPy equilibrium) are not solved: the platform stays at its
reference position, exactly the state the goldens are generated in.
"""
import ctypes

import numpy as np

from . import _native as N
from .fowt import FOWT
from .hydro_math import DEG2RAD, get_from_dict, wave_numbers
from .solver import CaseSet, solve_batch


class Model:
    def __init__(self, design, nTurbines=1, statics=None, device=0):
        """statics: optional per-FOWT dicts of calcStatics outputs (M_struc, C_struc, C_hydro,
        B_struc, W_struc, W_hydro) and C_moor; see FOWT.setStatics."""
        self.fowtList = []
        self.coords = []
        self.nDOF = 0
        if "settings" not in design:
            design["settings"] = {}
        st = design["settings"]
        min_freq = get_from_dict(st, "min_freq", default=0.01, dtype=float)
        max_freq = get_from_dict(st, "max_freq", default=1.00, dtype=float)
        self.XiStart = get_from_dict(st, "XiStart", default=0.1, dtype=float)
        self.nIter = get_from_dict(st, "nIter", default=15, dtype=int)
        self.w = self.frequency_grid(design)   # :55
        self.nw = len(self.w)
        self.depth = get_from_dict(design["site"], "water_depth", dtype=float)
        self.k = wave_numbers(self.w, self.depth)
        self.device = device
        self.K_array = None          # array-level mooring stiffness [6N,6N] (MoorPy in the reference)
        if "array" in design:
            self.nFOWT = len(design["array"]["data"])
            if "turbine" in design and "turbines" not in design:
                design["turbines"] = [design["turbine"]]
            if "platform" in design and "platforms" not in design:
                design["platforms"] = [design["platform"]]
            if "mooring" in design and "moorings" not in design:
                design["moorings"] = [design["mooring"]]
            info = [dict(zip(design["array"]["keys"], row)) for row in design["array"]["data"]]
            for i in range(self.nFOWT):
                d_i = {"site": design["site"]}
                if info[i]["turbineID"] != 0:
                    d_i["turbine"] = design["turbines"][info[i]["turbineID"] - 1]
                d_i["platform"] = design["platforms"][info[i]["platformID"] - 1]
                d_i["mooring"] = None if info[i]["mooringID"] == 0 else design["moorings"][info[i]["mooringID"] - 1]
                self.fowtList.append(FOWT(d_i, self.w, None, depth=self.depth, x_ref=info[i]["x_location"],
                                          y_ref=info[i]["y_location"], heading_adjust=info[i]["heading_adjust"],
                                          device=device))
                self.coords.append([info[i]["x_location"], info[i]["y_location"]])
                self.nDOF += 6
        else:
            self.nFOWT = 1
            self.fowtList.append(FOWT(design, self.w, None, depth=self.depth, device=device))
            self.coords.append([0.0, 0.0])
            self.nDOF += 6
        if statics is not None:
            for f, s in zip(self.fowtList, statics):
                f.setStatics(s)
        self.design = design
        self.results = {}

    @staticmethod
    def frequency_grid(design):
        """The first-order frequency grid [rad/s] of a design's settings (raft/raft_model.py:55)."""
        st = design.get("settings", {})
        min_freq = get_from_dict(st, "min_freq", default=0.01, dtype=float)
        max_freq = get_from_dict(st, "max_freq", default=1.00, dtype=float)
        return np.arange(min_freq, max_freq + 0.5 * min_freq, min_freq) * 2 * np.pi

    # --------------------------------------------------------------------- dynamics
    def solveDynamics(self, case, tol=0.01, conv_plot=0, RAO_plot=0, display=0):
        """raft/raft_model.py:852-1146 on the device.  Returns Xi [nWaves+1, 6N, nw] and sets
        fowt.Xi, fowt.Z, fowt.B_hydro_drag, fowt.F_hydro_drag, member Bmat like the reference.
        potSecOrder=1 FOWTs follow :966-989: first convergence -> RAO -> slender-body QTF ->
        second-order force -> a second drag pass from iteration 1 with the un-relaxed XiLast."""
        import torch
        iCase = case.get("iCase") if isinstance(case, dict) else None
        Zs, Fws = [], []
        for i, fowt in enumerate(self.fowtList):
            fowt.calcHydroExcitation(case, memberList=fowt.memberList)
            dd = fowt.device_design()
            dev = dd.device
            nW = fowt.nWaves
            fowt.Fhydro_2nd = np.zeros([nW, 6, self.nw], dtype=complex)
            fowt.Fhydro_2nd_mean = np.zeros([nW, 6])
            fowt._f2nd_w = [None] * nW
            cs = CaseSet([0], [case["wave_heading"][0]], [N.SPECTRUM_CODES[case["wave_spectrum"][0]]],
                         [case["wave_height"][0]], [case["wave_period"][0]], [case["wave_gamma"][0]])
            if display > 0:
                print("Solving for system response to wave excitation in primary wave direction")
            second = fowt.potSecOrder == 1
            want = ("zeta", "B_drag", "Bmat", "Z") + (("rao", "Xi_prev") if second else ())
            fext = None
            if fowt.potSecOrder == 2:   # external QTF: second-order load inside the drag loop (:903-904)
                fm, f = fowt.calcHydroForce_2ndOrd(fowt.beta[0], fowt._S_dev[0], iCase=iCase, iWT=i)
                fowt.Fhydro_2nd_mean[0], fowt.Fhydro_2nd[0] = fm, f
                fext = fowt._f2nd_dev.to(torch.complex128)[None].contiguous()
                fowt._f2nd_w[0] = fext[0]
            res = solve_batch([dd], cs, self.nIter, self.XiStart, tol, want=want, fext=fext)
            status, iters = self._check_pass(res, tol, display)
            fowt.iterations_pair = [iters]
            if second and status == N.RH_CASE_CONVERGED:
                if display > 1:
                    print("Resolving for system response in primary wave direction, now with second-order wave loads.")
                fowt.calcQTF_slenderBody(waveHeadInd=0, Xi0=res["rao"][0], verbose=True, iCase=iCase, iWT=i)
                fm, f = fowt.calcHydroForce_2ndOrd(fowt.beta[0], fowt._S_dev[0], iCase=iCase, iWT=i)
                fowt.Fhydro_2nd_mean[0], fowt.Fhydro_2nd[0] = fm, f
                fext = fowt._f2nd_dev.to(torch.complex128)[None].contiguous()
                fowt._f2nd_w[0] = fext[0]
                res = solve_batch([dd], cs, self.nIter, self.XiStart, tol, want=("zeta", "B_drag", "Bmat", "Z"),
                                  fext=fext, Xi_init=res["Xi_prev"].contiguous(), first_iter=1)
                status, iters = self._check_pass(res, tol, display)
                fowt.iterations_pair.append(iters)
            if status != N.RH_CASE_CONVERGED and display > 0:
                print("WARNING - solveDynamics iteration did not converge to the tolerance.")
            fowt.iterations, fowt.converged = iters, status == N.RH_CASE_CONVERGED
            Z = res["Z"][0]                                   # [nw,6,6]
            fowt.Z = np.moveaxis(Z.cpu().numpy(), 0, 2)
            fowt.B_hydro_drag = res["B_drag"][0].cpu().numpy()
            fowt._Bmat_dev = res["Bmat"][0].reshape(-1, 9).contiguous()
            fowt._scatter_bmat(fowt._Bmat_dev.cpu().numpy())
            Zs.append(Z)
            # excitation of every sea state with the final linearisation (:1049-1061)
            Fw = []
            for ih in range(nW):
                Fd = torch.tensor(fowt.calcDragExcitation(ih), dtype=torch.complex128, device=dev)
                if fowt.potSecOrder == 2 and ih > 0:                   # :1059-1060
                    fm, f = fowt.calcHydroForce_2ndOrd(fowt.beta[ih], fowt._S_dev[ih])
                    fowt.Fhydro_2nd_mean[ih], fowt.Fhydro_2nd[ih] = fm, f
                    fowt._f2nd_w[ih] = fowt._f2nd_dev.to(torch.complex128)
                F = dd.finer[fowt._heads[ih]] * fowt._zeta_dev[ih][None, :] + Fd
                if fowt._f2nd_w[ih] is not None:
                    F = F + fowt._f2nd_w[ih]
                Fw.append(F)
            Fws.append(Fw)
            fowt._res = res
        nW = self.fowtList[-1].nWaves           # the last FOWT's nWaves
        dev = self.fowtList[0].device_design().device
        Xi = torch.zeros([nW + 1, self.nDOF, self.nw], dtype=torch.complex128, device=dev)
        single = self.nFOWT == 1 and self.K_array is None
        for ih in range(nW):
            if single and ih == 0:
                Xi[0] = self.fowtList[0]._res["Xi"][0]                 # Zinv F_wave(0) == last solve
            else:
                Xi[ih] = self._system_solve(Zs, [Fw[ih] for Fw in Fws])
            # second-order loads of the other sea states (:1067-1083)
            if ih > 0 and any(f.potSecOrder == 1 for f in self.fowtList):
                for i, fowt in enumerate(self.fowtList):
                    if fowt.potSecOrder != 1:
                        continue
                    z = fowt._zeta_dev[ih]
                    x = Xi[ih, 6 * i:6 * i + 6]
                    rao = torch.where(z.abs() > 1e-6, x / torch.where(z == 0, torch.ones_like(z), z), torch.zeros_like(x))
                    fowt.calcQTF_slenderBody(waveHeadInd=ih, Xi0=rao, verbose=True, iCase=iCase, iWT=i)
                    fm, f = fowt.calcHydroForce_2ndOrd(fowt.beta[ih], fowt._S_dev[ih])
                    fowt.Fhydro_2nd_mean[ih], fowt.Fhydro_2nd[ih] = fm, f
                    Fws[i][ih] = Fws[i][ih] + fowt._f2nd_dev.to(torch.complex128)
                Xi[ih] = self._system_solve(Zs, [Fw[ih] for Fw in Fws])
        self.Xi = Xi.cpu().numpy()
        for i, fowt in enumerate(self.fowtList):
            xi_i = Xi[:, 6 * i:6 * i + 6, :].contiguous()
            psd = torch.empty([6, self.nw], dtype=torch.float64, device=dev)
            std = torch.empty([6], dtype=torch.float64, device=dev)
            N.check(N.lib().rh_motion_stats(N.context(self.device), 1, nW + 1, self.nw, float(fowt.dw), N.ptr(xi_i),
                                            N.ptr(psd), N.ptr(std), N.stream_handle(torch, dev)), "rh_motion_stats")
            fowt._stats = {"psd": psd.cpu().numpy(), "std": std.cpu().numpy()}
            fowt._xi_dev = xi_i                        # device copy for the derived channels
            fowt.Xi = self.Xi[:, 6 * i:6 * i + 6, :]
        self.results["response"] = {}
        return self.Xi

    @staticmethod
    def _check_pass(res, tol, display):
        """Status handling of one drag fixed point (raft/raft_model.py:954-966)."""
        iters = int(res["iters"].item())
        status = int(res["status"].item())
        if status == N.RH_CASE_NAN:
            raise Exception("Nan detected in response vector Xi.")
        if status == N.RH_CASE_SINGULAR:
            raise np.linalg.LinAlgError("Singular matrix")
        if display > 1 and status == N.RH_CASE_CONVERGED:
            print(f" Iteration {iters - 1}, converged (< {tol})")
        return status, iters

    def _system_solve(self, Zs, Fs):
        """Z_sys = blockdiag(Z_i) (+ K_array); Xi = Z_sys^-1 F (raft/raft_model.py:1021-1065)."""
        import torch
        dev = Zs[0].device
        nf = len(Zs)
        Z = torch.stack(Zs).contiguous()                  # [nf, nw, 6, 6]
        F = torch.cat(Fs, dim=0).contiguous()             # [6nf, nw]
        K = None
        if self.K_array is not None:
            K = torch.tensor(np.asarray(self.K_array, dtype=float), dtype=torch.float64, device=dev).contiguous()
        X = torch.empty([6 * nf, self.nw], dtype=torch.complex128, device=dev)
        N.check(N.lib().rh_system_solve(N.context(self.device), nf, self.nw, N.ptr(Z), N.ptr(K), N.ptr(F), N.ptr(X),
                                        N.stream_handle(torch, dev)), "rh_system_solve")
        return X

    # --------------------------------------------------------------------- cases
    def analyzeCases(self, display=0, meshDir=None, RAO_plot=False):
        """raft/raft_model.py:244-388 with the mean offsets held at the reference position."""
        nCases = len(self.design["cases"]["data"])
        self.results["properties"] = {}
        self.results["case_metrics"] = {}
        self.results["mean_offsets"] = []
        for fowt in self.fowtList:
            fowt.setPosition([fowt.x_ref, fowt.y_ref, 0, 0, 0, 0])
            fowt.calcStatics()
        for iCase in range(nCases):
            case = dict(zip(self.design["cases"]["keys"], self.design["cases"]["data"][iCase]))
            case["iCase"] = iCase
            self.results["case_metrics"][iCase] = {}
            for fowt in self.fowtList:
                fowt.calcTurbineConstants(case, ptfm_pitch=0)
                fowt.calcHydroConstants()
            self.solveDynamics(case, RAO_plot=RAO_plot, display=display)
            for i, fowt in enumerate(self.fowtList):
                self.results["case_metrics"][iCase][i] = {}
                fowt.saveTurbineOutputs(self.results["case_metrics"][iCase][i], case)
        return self.results

    def analyzeCasesBatch(self, cases, tol=0.01, want=("psd", "std", "zeta", "B_drag"), host=True):
        """Solve many single-sea-state cases of a single-FOWT model in one device call.
        cases: list of case dicts (wave_heading/spectrum/period/height/gamma).  Returns a dict
        of arrays: Xi [n,6,nw], iters, status, psd [n,6,nw], std [n,6], ..."""
        if self.nFOWT != 1:
            raise NotImplementedError("analyzeCasesBatch handles single-FOWT models")
        fowt = self.fowtList[0]
        hd, sp, Hs, Tp, gm = [], [], [], [], []
        for c in cases:
            c = dict(c)
            if not np.isscalar(c["wave_heading"]) and len(c["wave_heading"]) != 1:
                raise NotImplementedError("analyzeCasesBatch: one sea state per case")
            one = lambda k, dflt=None: (np.atleast_1d(c.get(k, dflt))[0] if c.get(k, dflt) is not None else None)
            hd.append(float(one("wave_heading", 0)))
            sp.append(str(one("wave_spectrum", "JONSWAP")))
            Hs.append(float(one("wave_height")))
            Tp.append(float(one("wave_period")))
            gm.append(float(one("wave_gamma", 0)))
        cs = CaseSet(np.zeros(len(cases), dtype=np.int32), hd, sp, Hs, Tp, gm)
        res = solve_batch([fowt.device_design()], cs, self.nIter, self.XiStart, tol, want=want)
        return res.host() if host else res
