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
from .fowt import FOWT, mooring_outputs
from .hydro_math import DEG2RAD, get_from_dict, wave_numbers
from .second_order import file_qtf_forces, qtf_index_error, solve_batch_2nd
from .solver import CaseSet, solve_batch


class CaseMB:
    """A per-case view of a DeviceDesign: the same node and wave tables, its own per-bin M and
    B [nw, 6, 6] device tensors (an operating rotor's aero-servo terms for one case)."""

    def __init__(self, base, M, B):
        self.base, self._M, self._B = base, M, B

    def __getattr__(self, name):
        return getattr(self.__dict__["base"], name)

    def ensure_headings(self, betas):
        return self.base.ensure_headings(betas)

    def struct(self):
        d = N.RhDesign.from_buffer_copy(self.base.struct())
        d.M, d.B, d.mb_per_bin = N.ptr(self._M), N.ptr(self._B), 1
        return d


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
        self.K_array = None          # array-level mooring stiffness override [6N,6N] (else from self.ms)
        self.ms = None               # array-level mooring system (raft/raft_model.py:83-102)
        if "array" in design:
            self.nFOWT = len(design["array"]["data"])
            if "turbine" in design and "turbines" not in design:
                design["turbines"] = [design["turbine"]]
            if "platform" in design and "platforms" not in design:
                design["platforms"] = [design["platform"]]
            if "mooring" in design and "moorings" not in design:
                design["moorings"] = [design["mooring"]]
            info = [dict(zip(design["array"]["keys"], row)) for row in design["array"]["data"]]
            if "array_mooring" in design:
                from .mooring import MooringSystem
                am = design["array_mooring"]
                if "file" not in am:
                    raise Exception("When using 'array_mooring', a MoorDyn-style input file must be provided as 'file'.")
                self.ms = MooringSystem(depth=self.depth)
                for i in range(self.nFOWT):
                    self.ms.add_body([info[i]["x_location"], info[i]["y_location"], 0, 0, 0, 0])
                self.ms.load_moordyn(am["file"])
            for i in range(self.nFOWT):
                d_i = {"site": design["site"]}
                if info[i]["turbineID"] != 0:
                    d_i["turbine"] = design["turbines"][info[i]["turbineID"] - 1]
                d_i["platform"] = design["platforms"][info[i]["platformID"] - 1]
                d_i["mooring"] = None if info[i]["mooringID"] == 0 else design["moorings"][info[i]["mooringID"] - 1]
                self.fowtList.append(FOWT(d_i, self.w, self.ms.bodies[i] if self.ms else None, depth=self.depth,
                                          x_ref=info[i]["x_location"],
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
        self.mooring_currentMod = get_from_dict(design.get("mooring") or {}, "currentMod", default=0, dtype=int)
        if self.ms is not None:
            self.ms.initialize()
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
        single = self.nFOWT == 1 and self.K_array is None and self.ms is None
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
        self._xi_dev_all = Xi
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

    def array_stiffness(self):
        """Array-level mooring stiffness added to Z_sys (raft/raft_model.py:1030-1031): the
        K_array override, else the array mooring system's analytic coupled stiffness."""
        if self.K_array is not None:
            return np.asarray(self.K_array, dtype=float)
        if self.ms is not None:
            return self.ms.coupled_stiffness_analytic()
        return None

    def _system_solve(self, Zs, Fs):
        """Z_sys = blockdiag(Z_i) (+ K_array); Xi = Z_sys^-1 F (raft/raft_model.py:1021-1065)."""
        import torch
        dev = Zs[0].device
        nf = len(Zs)
        Z = torch.stack(Zs).contiguous()                  # [nf, nw, 6, 6]
        F = torch.cat(Fs, dim=0).contiguous()             # [6nf, nw]
        K = None
        Ka = self.array_stiffness()
        if Ka is not None:
            K = torch.tensor(Ka, dtype=torch.float64, device=dev).contiguous()
        X = torch.empty([6 * nf, self.nw], dtype=torch.complex128, device=dev)
        N.check(N.lib().rh_system_solve(N.context(self.device), nf, self.nw, N.ptr(Z), N.ptr(K), N.ptr(F), N.ptr(X),
                                        N.stream_handle(torch, dev)), "rh_system_solve")
        return X

    # --------------------------------------------------------------------- statics
    def solveStatics(self, case, display=0):
        """Mean offsets of every FOWT for a load case (raft/raft_model.py:479-790): linear
        hydrostatics about the reference position (statics_mod 0), constant environmental
        loads (forcing_mod 0: mean aero = 0 here, current drag, mean wave drift), nonlinear
        mooring forces, Newton steps on the total stiffness through dsolve2.  Leaves every
        FOWT at its offset pose (setPosition), as the reference does."""
        from .dsolve import dsolve2
        nD = self.nDOF
        K_hs, F_und = [], np.zeros(nD)
        F_env = np.zeros(nD)
        X_init = np.zeros(nD)
        if case and isinstance(case.get("wind_speed"), list) and len(case["wind_speed"]) != len(self.fowtList):
            raise IndexError("List of wind speeds must be the same length as the list of wind turbines")
        for i, fowt in enumerate(self.fowtList):
            X_init[6 * i:6 * i + 6] = [fowt.x_ref, fowt.y_ref, 0, 0, 0, 0]
            fowt.setPosition(X_init[6 * i:6 * i + 6])
            fowt.calcStatics()
            K_hs.append(fowt.C_struc + fowt.C_hydro)
            F_und[6 * i:6 * i + 6] += fowt.W_struc + fowt.W_hydro
            if case:
                ci = dict(case)
                if isinstance(case.get("wind_speed"), list):
                    ci["wind_speed"] = case["wind_speed"][i]
                fowt.calcTurbineConstants(ci, ptfm_pitch=0)
                fowt.calcHydroConstants()
                F_env[6 * i:6 * i + 6] = np.sum(fowt.f_aero0, axis=1) + fowt.calcCurrentLoads(ci)
                if getattr(fowt, "Fhydro_2nd_mean", None) is not None:
                    F_env[6 * i:6 * i + 6] += np.sum(fowt.Fhydro_2nd_mean, axis=0)
        # uniform current on the mooring lines (raft/raft_model.py:561-577): set for this case,
        # cleared otherwise, on the array system and every FOWT's own system
        cur = np.zeros(3)
        if case and self.mooring_currentMod > 0:
            speed = get_from_dict(case, "current_speed", shape=0, default=0.0)
            head = get_from_dict(case, "current_heading", shape=0, default=0)
            if speed > 0:
                cur = np.array([speed * np.cos(np.radians(head)), speed * np.sin(np.radians(head)), 0.0])
        for sysm in [self.ms] + [fowt.ms for fowt in self.fowtList]:
            if sysm is not None:
                sysm.current = cur.copy()
        tols = np.array([0.05, 0.05, 0.05, 0.005, 0.005, 0.005] * len(self.fowtList))

        def eval_func(X, args):
            for i, fowt in enumerate(self.fowtList):
                fowt.setPosition(X[6 * i:6 * i + 6])
            if self.ms is not None:
                self.ms.set_body_positions([X[6 * i:6 * i + 6] for i in range(self.nFOWT)])
            Fnet = np.zeros(nD)
            for i, fowt in enumerate(self.fowtList):
                Xi0 = X[6 * i:6 * i + 6] - np.array([fowt.x_ref, fowt.y_ref, 0, 0, 0, 0])
                Fnet[6 * i:6 * i + 6] += F_und[6 * i:6 * i + 6]
                Fnet[6 * i:6 * i + 6] += -np.matmul(K_hs[i], Xi0)
                if case:
                    Fnet[6 * i:6 * i + 6] += F_env[6 * i:6 * i + 6]
                Fnet[6 * i:6 * i + 6] += fowt.F_moor0
                if self.ms is not None:
                    Fnet[6 * i:6 * i + 6] += self.ms.body_forces(self.ms.bodies[i], lines_only=True)
            return Fnet, dict(status=1), False

        def step_func(X, args, Y, oths, Ytarget, err, tol_, it, maxIter):
            K = np.zeros([nD, nD])
            if self.ms is not None:
                K += self.ms.coupled_stiffness_analytic()
            for i, fowt in enumerate(self.fowtList):
                K6 = K_hs[i].copy()
                if fowt.ms is not None:
                    K6 += fowt.ms.coupled_stiffness_analytic()
                K[6 * i:6 * i + 6, 6 * i:6 * i + 6] += K6
            kmean = np.mean(K.diagonal())
            for i in range(nD):
                if K[i, i] == 0:
                    K[i, i] = kmean
            dX = np.linalg.solve(K, Y)
            for _ in range(10):                       # strengthen the diagonal on a backward step (:738-748)
                if sum(dX * Y) < 0:
                    for i in range(nD):
                        K[i, i] += 0.1 * abs(K[i, i])
                    dX = np.linalg.solve(K, Y)
                else:
                    break
            return dX

        X, Y, info = dsolve2(eval_func, X_init, step_func=step_func, tol=tols, a_max=1.6, maxIter=20,
                             args={"display": display})
        self.Xs2, self.Es2 = info["Xs"], info["Es"]
        if case and "iCase" in case:
            self.results.setdefault("mean_offsets", []).append(self.Xs2[-1])
        if display > 0:
            for i, fowt in enumerate(self.fowtList):
                print(f"Found mean offets of FOWT {i + 1} with surge = {fowt.Xi0[0]: .2f} m,  sway  = "
                      f"{fowt.Xi0[1]: .2f},  and heave = {fowt.Xi0[2]: .2f} m")
        return X

    def solveEigen(self, display=0):
        """Natural frequencies [Hz] and mode shapes of the moored system
        (raft/raft_model.py:391-476): M = M_struc + A_hydro_morison, C = C_struc + C_hydro +
        C_moor (+ yaw stiffness, + array mooring).  Host LAPACK on a 6N x 6N pencil."""
        nD = self.nDOF
        M_tot = np.zeros([nD, nD])
        C_tot = np.zeros([nD, nD])
        for i, fowt in enumerate(self.fowtList):
            i1, i2 = 6 * i, 6 * i + 6
            M_tot[i1:i2, i1:i2] += fowt.M_struc + fowt.A_hydro_morison
            C_tot[i1:i2, i1:i2] += fowt.C_struc + fowt.C_hydro + fowt.C_moor
            C_tot[i1 + 5, i1 + 5] += fowt.yawstiff
        if self.ms is not None:
            C_tot += self.ms.coupled_stiffness_analytic()
        message = ""
        for i in range(nD):
            if M_tot[i, i] < 1.0:
                message += f"Diagonal entry {i} of system mass matrix is less than 1 ({M_tot[i, i]}). "
            if C_tot[i, i] < 1.0:
                message += f"Diagonal entry {i} of system stiffness matrix is less than 1 ({C_tot[i, i]}). "
        if message:
            raise RuntimeError("System matrices computed by RAFT have one or more small or negative diagonals: "
                               + message)
        eigenvals, eigenvectors = np.linalg.eig(np.linalg.solve(M_tot, C_tot))
        if any(eigenvals <= 0.0):
            raise RuntimeError("Error: zero or negative system eigenvalues detected.")
        ind_list = []
        for i in range(nD - 1, -1, -1):              # DOF order by the largest mode component (:442-456)
            vec = np.abs(eigenvectors[i, :])
            for _ in range(nD):
                ind = np.argmax(vec)
                if ind in ind_list:
                    vec[ind] = 0.0
                else:
                    ind_list.append(ind)
                    break
        ind_list.reverse()
        fns = np.sqrt(eigenvals[ind_list]) / 2.0 / np.pi
        modes = eigenvectors[:, ind_list]
        if display > 0:
            print("Fn (Hz)" + "".join([f"{fn:10.4f}" for fn in fns]))
        self.results["eigen"] = {"frequencies": fns, "modes": modes}
        return fns, modes

    def analyzeUnloaded(self, ballast=0, heave_tol=1):
        """Unloaded equilibrium and mooring properties (raft/raft_model.py:184-241)."""
        if len(self.fowtList) > 1:
            raise Exception("analyzeUnloaded is an old method that only works for a single FOWT.")
        if ballast:
            raise NotImplementedError("ballast adjustment (raft/raft_model.py:1434-1625) is outside the accelerated path")
        f0 = self.fowtList[0]
        f0.setPosition(np.zeros(6))
        f0.D_hydr0 = np.zeros(6)
        f0.f_aero0 = np.zeros([6, f0.nrotors])
        self.C_moor0 = np.zeros([6, 6])
        self.F_moor0 = np.zeros(6)
        for ms in (self.ms, f0.ms):
            if ms is not None:
                self.C_moor0 += ms.coupled_stiffness_fd()
                self.F_moor0 += ms.coupled_forces(lines_only=True)
        for fowt in self.fowtList:
            fowt.calcStatics()
            fowt.calcHydroConstants()
        self.results["properties"] = {}
        self.solveStatics(None)
        self.results["properties"]["offset_unloaded"] = self.fowtList[0].Xi0

    def calcOutputs(self):
        """System property outputs of the first FOWT (raft/raft_model.py:1150-1189)."""
        fowt = self.fowtList[0]
        if "properties" in self.results:
            C0 = getattr(self, "C_moor0", np.zeros([6, 6]))
            P = self.results["properties"]
            P["tower mass"] = fowt.mtower
            P["tower CG"] = fowt.rCG_tow
            P["substructure mass"] = fowt.m_sub
            P["substructure CG"] = fowt.rCG_sub
            P["shell mass"] = fowt.m_shell
            P["ballast mass"] = fowt.m_ballast
            P["ballast densities"] = fowt.pb
            P["total mass"] = fowt.M_struc[0, 0]
            P["total CG"] = fowt.rCG
            P["roll inertia at subCG"] = fowt.props["Ixx_sub"]
            P["pitch inertia at subCG"] = fowt.props["Iyy_sub"]
            P["yaw inertia at subCG"] = fowt.props["Izz_sub"]
            P["buoyancy (pgV)"] = fowt.rho_water * fowt.g * fowt.V
            P["center of buoyancy"] = fowt.rCB
            P["C hydrostatic"] = fowt.C_hydro
            P["C system"] = fowt.C_struc + fowt.C_hydro + C0
            P["F_lines0"] = getattr(self, "F_moor0", np.zeros(6))
            P["C_lines0"] = C0
            P["M support structure"] = fowt.M_struc_sub
            P["A support structure"] = fowt.A_hydro_morison + fowt.A_BEM[:, :, -1]
            P["C support structure"] = fowt.C_struc_sub + fowt.C_hydro + C0
        return self.results

    # --------------------------------------------------------------------- cases
    def analyzeCases(self, display=0, meshDir=None, RAO_plot=False):
        """raft/raft_model.py:244-388: per case, mean offsets (solveStatics), the response
        solve on the device, and the output channels of every FOWT (plus array-level mooring
        tensions).  When every FOWT's mooring stiffness was given as a fixture (setStatics with a
        C_moor, e.g. the reference-run goldens), the platforms stay at their reference position."""
        nCases = len(self.design["cases"]["data"])
        self.results["properties"] = {}
        self.results["case_metrics"] = {}
        self.results["mean_offsets"] = []
        for fowt in self.fowtList:
            fowt.setPosition([fowt.x_ref, fowt.y_ref, 0, 0, 0, 0])
            fowt.calcStatics()
        for iCase in range(nCases):
            if display > 0:
                print(f"\n--------------------- Running Case {iCase + 1} ----------------------")
                print(self.design["cases"]["data"][iCase])
            case = dict(zip(self.design["cases"]["keys"], self.design["cases"]["data"][iCase]))
            case["iCase"] = iCase
            nWaves = 1 if np.isscalar(case["wave_heading"]) else len(case["wave_heading"])
            self.results["case_metrics"][iCase] = {}
            fixture = all("C_moor" in (f._statics or {}) for f in self.fowtList)
            if fixture:       # mooring given as a stiffness fixture (setStatics): positions held at the reference
                for fowt in self.fowtList:
                    fowt.calcTurbineConstants(case, ptfm_pitch=0)
                    fowt.calcHydroConstants()
            else:
                self.solveStatics(case, display=display)
            self.solveDynamics(case, RAO_plot=RAO_plot, display=display)
            if any(f.potSecOrder > 0 for f in self.fowtList):
                if not fixture:
                    self.solveStatics(case)
                for fowt in self.fowtList:
                    fowt.Fhydro_2nd_mean *= 0
            for i, fowt in enumerate(self.fowtList):
                self.results["case_metrics"][iCase][i] = {}
                fowt.saveTurbineOutputs(self.results["case_metrics"][iCase][i], case)
            if self.ms is not None:
                self.results["case_metrics"][iCase]["array_mooring"] = mooring_outputs(
                    self.ms, self._xi_dev_all, self.w, self.device, nWaves + 1)
        return self.results

    def analyzeCasesBatch(self, cases, tol=0.01, want=("psd", "std", "zeta", "B_drag"), host=True):
        """Solve many cases in one device call (one workgroup per case's drag fixed point).
        cases: list of case dicts (wave_heading/spectrum/period/height/gamma, each a scalar or
        one entry per sea state; with wind_speed > 0 on an operating rotor, that case's
        aero-servo M and B from calcTurbineConstants).  Returns a dict of arrays: Xi [n,6,nw]
        (the first sea state), iters, status, psd [n,6,nw], std [n,6], ...
        A case with several sea states is solved as Model.solveDynamics solves it
        (raft/raft_model.py:918-1065): the drag linearisation from its first sea state, then the
        response to each sea state with that linearisation frozen (one rh_heading_response launch
        for every extra sea state of the batch); Xi_waves [n, nW+1, 6, nw] holds them in the
        reference's layout (nW = the batch's largest sea-state count, rows of absent sea states
        and the last row zero) and psd / std sum over the sea states (getPSD / getRMS).
        Second-order loads (raft/raft_model.py:899-1083) as solveDynamics applies them
        (raft/second_order.py): potSecOrder=2 adds the .12d QTF's force of every sea state
        (f2nd_mean [n,6] of sea state 0, f2nd_mean_waves [n,nW,6] with several sea states);
        potSecOrder=1 solves twice, the QTF of each converged case's RAO between the passes
        (iters_pair [n,2]); several sea states per case raise the reference's IndexError (Q8).
        Arrays (nFOWT > 1) go through analyzeArrayBatch: Xi [n,6N,nw], iters [n,N], ..."""
        if self.nFOWT != 1:
            return self.analyzeArrayBatch(cases, tol=tol, host=host)
        fowt = self.fowtList[0]
        seas = [self._case_sea_states(c) for c in cases]
        nws = np.array([len(s[0]) for s in seas], dtype=np.int64)
        if fowt.potSecOrder == 1 and len(cases) and nws.max() > 1:
            raise qtf_index_error(1)      # the slender-body QTF of sea state 1
        hd, sp, Hs, Tp, gm = ([s[k][0] for s in seas] for k in range(5))
        multi = len(cases) > 0 and nws.max() > 1
        want_fp = tuple(want) + (("Bmat", "B_drag") if multi else ())
        aero = [self._operating_rotor(fowt, c) for c in cases]
        if multi:   # every heading tabulated before the fixed point (its tables stay put)
            fowt.device_design().ensure_headings(np.concatenate([np.asarray(s[0], dtype=float) for s in seas]) * DEG2RAD)
        if not any(aero):
            views = [fowt.device_design()]
            cs = CaseSet(np.zeros(len(cases), dtype=np.int32), hd, sp, Hs, Tp, gm)
            res = solve_batch_2nd(views, [fowt], cs, self.nIter, self.XiStart, tol, want=want_fp)
            if multi:
                self._extra_sea_states(res, views, cs.design_idx, seas, nws, want)
            return res.host() if host else res
        # operating rotors: each such case gets its own per-bin M and B (its rotors' aero-servo
        # added mass and damping, FOWT.calcTurbineConstants) on the shared node and wave tables
        import torch
        from .prep import linear_matrices
        fowt.calcTurbineConstants(dict(cases[0], wind_speed=0.0), ptfm_pitch=0)     # the aero-free design
        base = fowt.device_design()
        base.ensure_headings(np.unique(np.asarray(hd, dtype=float)) * DEG2RAD)
        views, idx = [base], np.zeros(len(cases), dtype=np.int32)
        for i, c in enumerate(cases):
            if aero[i]:
                fowt.calcTurbineConstants(dict(c), ptfm_pitch=0)
                M, B, _, _ = linear_matrices(fowt)
                f64 = dict(dtype=torch.float64, device=base.device)
                views.append(CaseMB(base, torch.tensor(M, **f64).contiguous(), torch.tensor(B, **f64).contiguous()))
                idx[i] = len(views) - 1
        cs = CaseSet(idx, hd, sp, Hs, Tp, gm)
        res = solve_batch_2nd(views, [fowt] * len(views), cs, self.nIter, self.XiStart, tol, want=want_fp)
        if multi:
            self._extra_sea_states(res, views, idx, seas, nws, want)
        return res.host() if host else res

    @staticmethod
    def _case_sea_states(case):
        """The sea states of one case dict, read as FOWT.calcHydroExcitation reads them
        (raft/raft_fowt.py:982-1014): (heading [deg], spectrum, Hs, Tp, gamma), one entry each
        per sea state."""
        c = dict(case)
        hd = c.get("wave_heading", 0)
        nW = 1 if np.isscalar(hd) else len(hd)
        col = lambda k, **kw: list(np.atleast_1d(get_from_dict(c, k, shape=nW, **kw)))   # noqa: E731
        sp = [str(x) for x in col("wave_spectrum", dtype=str, default="JONSWAP")]
        for x in sp:
            if x not in N.SPECTRUM_CODES:
                raise ValueError(f"Wave spectrum input '{x}' not recognized.")
        return ([float(x) for x in col("wave_heading", dtype=float, default=0)], sp,
                [float(x) for x in col("wave_height", dtype=float)], [float(x) for x in col("wave_period", dtype=float)],
                [float(x) for x in col("wave_gamma", dtype=float, default=0)])

    def _extra_sea_states(self, res, views, idx, seas, nws, want):
        """The response of every case's further sea states with its drag linearisation frozen
        (raft/raft_model.py:1049-1065): their spectra (rh_sea_state), one rh_heading_response
        launch for all of them, Xi_waves [n, nW+1, 6, nw] and psd / std over all sea states
        (rh_motion_stats, getPSD / getRMS of raft/raft_fowt.py:1831-1875)."""
        import torch
        n, nw = len(seas), self.nw
        nwm = int(nws.max())
        dd = views[0]
        dev = dd.device
        i32 = dict(dtype=torch.int32, device=dev)
        f64 = dict(dtype=torch.float64, device=dev)
        ext = [(i, h) for i in range(n) for h in range(1, int(nws[i]))]
        ci = np.array([i for i, _ in ext], dtype=np.int64)
        pick = lambda k: [seas[i][k][h] for i, h in ext]   # noqa: E731
        betas = np.array(pick(0), dtype=float) * DEG2RAD
        heads = dd.ensure_headings(betas)
        ctx, s = N.context(self.device), N.stream_handle(torch, dev)
        m = len(ext)
        S = torch.empty([m, nw], **f64)
        zeta = torch.empty([m, nw], **f64)
        spec = torch.tensor([N.SPECTRUM_CODES[x] for x in pick(1)], **i32)
        Hs, Tp, gm = (torch.tensor(pick(k), **f64) for k in (2, 3, 4))
        N.check(N.lib().rh_sea_state(ctx, m, nw, N.ptr(dd.w), float(dd.dw), N.ptr(spec), N.ptr(Hs), N.ptr(Tp),
                                     N.ptr(gm), N.ptr(S), N.ptr(zeta), s), "rh_sea_state")
        sel = torch.tensor(ci, dtype=torch.long, device=dev)
        bdrag = res["B_drag"].index_select(0, sel).contiguous()
        bmat = res["Bmat"].index_select(0, sel).contiguous()
        XiE = torch.empty([m, 6, nw], dtype=torch.complex128, device=dev)
        fext = None
        fowt = self.fowtList[0]
        if fowt.potSecOrder == 2:      # the .12d QTF's force of each further sea state (:1059-1061)
            fext, fm = file_qtf_forces(dd, fowt, betas, S)
            fw = torch.zeros([n, nwm, 6], **f64)
            fw[:, 0] = res["f2nd_mean"]
            fw[sel, torch.tensor([h for _, h in ext], dtype=torch.long, device=dev)] = fm
            res["f2nd_mean_waves"] = fw
        arr = (N.RhDesign * len(views))(*[v.struct() for v in views])
        # (the index tensors are held in names: a temporary freed before the call returns would
        # hand its block to the next allocation, and the kernel would read the other array)
        didx = torch.tensor(np.asarray(idx)[ci], **i32)
        hidx = torch.tensor(heads, **i32)
        N.check(N.lib().rh_heading_response_ext(ctx, arr, len(views), m, N.ptr(didx), N.ptr(hidx), N.ptr(zeta),
                                                N.ptr(bdrag), N.ptr(bmat), int(bmat.shape[1]), N.ptr(fext), N.ptr(XiE),
                                                s), "rh_heading_response_ext")
        Xw = torch.zeros([n, nwm + 1, 6, nw], dtype=torch.complex128, device=dev)
        Xw[:, 0] = res["Xi"]
        Xw[sel, torch.tensor([h for _, h in ext], dtype=torch.long, device=dev)] = XiE
        res["Xi_waves"] = Xw
        if "psd" in want or "std" in want:
            psd = torch.empty([n, 6, nw], **f64)
            std = torch.empty([n, 6], **f64)
            N.check(N.lib().rh_motion_stats(ctx, n, nwm + 1, nw, float(dd.dw), N.ptr(Xw), N.ptr(psd), N.ptr(std), s),
                    "rh_motion_stats")
            res["psd"], res["std"] = psd, std
        res["nWaves"] = torch.tensor(nws, dtype=torch.int64, device=dev)

    @staticmethod
    def _operating_rotor(fowt, case):
        """Whether calcTurbineConstants gives this case aero terms (raft/raft_fowt.py:795-812).
        A batch case without a wind_speed entry is a sea state alone (wind 0), as batch cases
        have always been read here."""
        if fowt.nrotors == 0:
            return False
        status = get_from_dict(case, "turbine_status", shape=0, dtype=str, default="operating")
        speed = get_from_dict(case, "wind_speed", shape=0, default=0.0)
        return status == "operating" and speed > 0.0 and bool(np.any(np.atleast_1d(fowt._aero_mod) > 0))

    def prepareArrayBatch(self, cases):
        """The per-batch inputs of analyzeArrayBatch resident on the device: the (case, FOWT)
        case table with its wave tables (solver.prepare_batch), the FOWT descriptors and the
        array stiffness.  Reusable for repeated solves of the same sea states.  Every heading of
        every sea state is tabulated here, before any descriptor is made."""
        import torch
        nf, n = self.nFOWT, len(cases)
        dds = [f.device_design() for f in self.fowtList]   # (node counts may differ: Bmat rows padded to the largest)
        seas = [self._case_sea_states(c) for c in cases]
        nws = np.array([len(x[0]) for x in seas], dtype=np.int64)
        if any(f.potSecOrder == 1 for f in self.fowtList):
            raise NotImplementedError("analyzeArrayBatch: potSecOrder=1 in a coupled array; the reference adds the "
                                      "force to F_lin[i1:i2] of the whole system (raft/raft_model.py:988, SURVEY.md Q5)")
        allh = np.unique(np.concatenate([np.asarray(x[0], dtype=float) for x in seas])) * DEG2RAD if n else []
        for d in dds:
            d.ensure_headings(allh)
        hd, sp, Hs, Tp, gm = ([x[k][0] for x in seas] for k in range(5))
        rep = lambda v: [x for x in v for _ in range(nf)]          # case-major, FOWT-minor
        cs = CaseSet(np.tile(np.arange(nf, dtype=np.int32), n), rep(hd), rep(sp), rep(Hs), rep(Tp), rep(gm))
        dev = dds[0].device
        from .solver import prepare_batch
        Ka = self.array_stiffness()
        return dict(n=n, dds=dds, cs=cs, prep=prepare_batch(dds, cs), dev=dev, seas=seas, nws=nws,
                    arr=(N.RhDesign * nf)(*[d.struct() for d in dds]),
                    K=None if Ka is None else torch.tensor(Ka, dtype=torch.float64, device=dev).contiguous())

    def analyzeArrayBatch(self, cases=None, tol=0.01, host=True, marks=None, prepared=None):
        """The coupled-array response of many cases (raft/raft_model.py:852-1065 for nFOWT > 1)
        in a few device calls instead of per-case, per-FOWT host round trips:
          1. every (case, FOWT) drag fixed point in one rh_solve_cases launch (outputs: zeta,
             the node drag matrices, B_drag, and each entry's wave excitation of sea state 0
             with its final linearisation, F_wave);
          2. rh_array_solve_stats: per (case, bin) each FOWT's impedance rebuilt from the
             design's matrices and B_drag, Z_sys = blockdiag(Z_i) + array mooring stiffness and
             Xi = Z_sys^-1 F_wave, and the per-FOWT motion PSD / RMS from the solution in
             registers (rh_motion_stats' values, bit for bit);
          3. cases with several sea states (:1049-1065): the excitation of every further
             (sea state, FOWT) with the linearisation frozen (rh_wave_excitation) and the same
             coupled solve for all of them in one more launch; psd / std then sum over the sea
             states (rh_motion_stats over Xi_waves, getPSD / getRMS) and Xi_waves
             [n, nW+1, 6N, nw] holds every response in the reference's layout.
        FOWTs with potSecOrder=2 add their .12d QTF's force to each sea state's excitation
        (:903-904, :1059-1061; f2nd_mean [n, N, 6]).
        Returns Xi [n, 6N, nw], iters / status [n, N], psd [n, N, 6, nw], std [n, N, 6], zeta.
        prepared: prepareArrayBatch(cases) of an earlier call (then `cases` is not needed).
        marks: optional two timing events recorded around the fixed-point launch (bench)."""
        import torch
        P = prepared if prepared is not None else self.prepareArrayBatch(cases)
        nf, n, nw = self.nFOWT, P["n"], self.nw
        dds, cs, prep, dev = P["dds"], P["cs"], P["prep"], P["dev"]
        multi = n > 0 and int(P["nws"].max()) > 1
        # X first holds each (case, FOWT)'s F_wave, written by its fixed point with the final
        # linearisation ([n, 6 nf, nw] is the [n nf, 6, nw] layout of the fixed point's entries),
        # then the coupled response (rh_array_solve_stats)
        X = torch.empty([n, 6 * nf, nw], dtype=torch.complex128, device=dev)
        if marks:
            marks[0].record(torch.cuda.current_stream(dev))
        res = solve_batch_2nd(dds, self.fowtList, cs, self.nIter, self.XiStart, tol,
                              want=("zeta", "Bmat", "B_drag", "noXi"), prepared=prep, F_wave=X.view(n * nf, 6, nw))
        if marks:
            marks[1].record(torch.cuda.current_stream(dev))
        arr = P["arr"]
        s = N.stream_handle(torch, dev)
        ctx = N.context(self.device)
        K = P["K"]
        psd = std = None
        if not multi:
            psd = torch.empty([n * nf, 6, nw], dtype=torch.float64, device=dev)
            std = torch.empty([n * nf, 6], dtype=torch.float64, device=dev)
        N.check(N.lib().rh_array_solve_stats(ctx, arr, nf, nf, n, N.ptr(prep["design"]), N.ptr(res["B_drag"]), N.ptr(K),
                                             N.ptr(X), float(self.fowtList[0].dw), N.ptr(psd), N.ptr(std), s),
                "rh_array_solve_stats")
        out = {"Xi": X, "iters": res["iters"].view(n, nf), "status": res["status"].view(n, nf),
               "zeta": res["zeta"].view(n, nf, nw)[:, 0]}
        if "f2nd_mean" in res:
            out["f2nd_mean"] = res["f2nd_mean"].view(n, nf, 6)
        keep = [res, arr, K]
        if multi:
            psd, std = self._array_extra_sea_states(P, res, X, out, keep)
        out["psd"], out["std"] = psd.view(n, nf, 6, nw), std.view(n, nf, 6)
        out["_keep"] = tuple(keep)
        if host:
            return {k: v.cpu().numpy() for k, v in out.items() if k != "_keep"}
        return out

    def _array_extra_sea_states(self, P, res, X, out, keep):
        """Step 3 of analyzeArrayBatch: the further sea states of every case (one excitation and
        one coupled-solve launch for all of them), Xi_waves and the statistics over all rows."""
        import torch
        nf, n, nw = self.nFOWT, P["n"], self.nw
        dds, dev, seas, nws = P["dds"], P["dev"], P["seas"], P["nws"]
        nwm = int(nws.max())
        ctx, s = N.context(self.device), N.stream_handle(torch, dev)
        i32 = dict(dtype=torch.int32, device=dev)
        f64 = dict(dtype=torch.float64, device=dev)
        ext = [(i, h) for i in range(n) for h in range(1, int(nws[i]))]
        m = len(ext)
        pick = lambda k: [seas[i][k][h] for i, h in ext]   # noqa: E731
        betas = np.array(pick(0), dtype=float) * DEG2RAD
        from .second_order import sea_spectra
        S, zeta = sea_spectra(dds[0], [N.SPECTRUM_CODES[x] for x in pick(1)], pick(2), pick(3), pick(4))
        # entries (extra sea state, FOWT), sea-state-major: the [m, 6 nf, nw] layout of the solve
        src = np.array([i * nf + f for i, _ in ext for f in range(nf)], dtype=np.int64)
        heads = np.array([dds[f].ensure_headings([b])[0] for b in betas for f in range(nf)], dtype=np.int32)
        didx = torch.tensor(np.tile(np.arange(nf, dtype=np.int32), m), **i32)
        hidx = torch.tensor(heads, **i32)
        srct = torch.tensor(src, dtype=torch.long, device=dev)
        ze = zeta.repeat_interleave(nf, dim=0).contiguous()
        bmat = res["Bmat"].index_select(0, srct).contiguous()
        bdrag = res["B_drag"].index_select(0, srct).contiguous()
        XE = torch.empty([m, 6 * nf, nw], dtype=torch.complex128, device=dev)
        N.check(N.lib().rh_wave_excitation(ctx, P["arr"], nf, m * nf, N.ptr(didx), N.ptr(hidx), N.ptr(ze), N.ptr(bmat),
                                           N.ptr(XE), s), "rh_wave_excitation")
        FE = XE.view(m, nf, 6, nw)
        if any(f.potSecOrder == 2 for f in self.fowtList):
            fw = torch.zeros([n, nwm, nf, 6], **f64)
            fw[:, 0] = out["f2nd_mean"]
            hsel = torch.tensor([h for _, h in ext], dtype=torch.long, device=dev)
            csel = torch.tensor([i for i, _ in ext], dtype=torch.long, device=dev)
            for f, fowt in enumerate(self.fowtList):
                if fowt.potSecOrder != 2:
                    continue
                fx, fm = file_qtf_forces(dds[f], fowt, betas, S)          # (:1059-1061)
                FE[:, f] += fx
                fw[csel, hsel, f] = fm
            out["f2nd_mean_waves"] = fw
        N.check(N.lib().rh_array_solve_stats(ctx, P["arr"], nf, nf, m, N.ptr(didx), N.ptr(bdrag), N.ptr(P["K"]),
                                             N.ptr(XE), float(self.fowtList[0].dw), None, None, s),
                "rh_array_solve_stats")
        Xw = torch.zeros([n, nwm + 1, 6 * nf, nw], dtype=torch.complex128, device=dev)
        Xw[:, 0] = X
        Xw[torch.tensor([i for i, _ in ext], dtype=torch.long, device=dev),
           torch.tensor([h for _, h in ext], dtype=torch.long, device=dev)] = XE
        out["Xi_waves"] = Xw
        out["nWaves"] = torch.tensor(nws, dtype=torch.int64, device=dev)
        rows = Xw.view(n, nwm + 1, nf, 6, nw).permute(0, 2, 1, 3, 4).contiguous()      # [n, nf, nW+1, 6, nw]
        psd = torch.empty([n * nf, 6, nw], **f64)
        std = torch.empty([n * nf, 6], **f64)
        N.check(N.lib().rh_motion_stats(ctx, n * nf, nwm + 1, nw, float(self.fowtList[0].dw), N.ptr(rows), N.ptr(psd),
                                        N.ptr(std), s), "rh_motion_stats")
        keep += [S, zeta, didx, hidx, ze, bmat, bdrag, XE, rows]
        return psd, std


def _load_design(input_file):
    """A design dict from a dict or a YAML file (raft/raft_model.py:2029-2039).  Pickled
    designs are refused: unpickling can execute code from the file."""
    if isinstance(input_file, dict):
        return input_file
    if str(input_file).endswith((".pkl", ".pickle")):
        raise ValueError("pickled design files are not loaded (unpickling can execute code); pass a YAML file or a dict")
    import yaml
    print("\n\nLoading RAFT input file: " + str(input_file))
    with open(input_file) as fh:
        return yaml.safe_load(fh)


def runRAFT(input_file, turbine_file="", plot=0, ballast=False, station_plot=[]):
    """Set up and run RAFT for a design (raft/raft_model.py:2024-2061): Model, unloaded
    equilibrium, every load case of design['cases'] (mean offsets, device response solve,
    output channels) and the system property outputs.  Returns the Model."""
    design = _load_design(input_file)
    print(" --- making model ---")
    model = Model(design)
    print(" --- analyzing unloaded ---")
    model.analyzeUnloaded(ballast=ballast)
    print(" --- analyzing cases ---")
    model.analyzeCases(display=1)
    model.calcOutputs()
    if plot:
        raise NotImplementedError("plotting is outside the accelerated path")
    return model


def runRAFTFarm(input_file, plot=0):
    """Set up and run a RAFT farm (raft/raft_model.py:2065-2095): no unloaded analysis and no
    calcOutputs (as in the reference); analyzeCases over the coupled array."""
    design = _load_design(input_file)
    print(" --- making model ---")
    model = Model(design)
    print("**Note: RAFTFarm cannot run model.analyzeUnloaded()")
    print(" --- analyzing cases ---")
    model.analyzeCases(display=1)
    print("**Note: model.calcOutputs is not supported yet for multi-turbine Farm configurations")
    if plot:
        raise NotImplementedError("plotting is outside the accelerated path")
    return model
