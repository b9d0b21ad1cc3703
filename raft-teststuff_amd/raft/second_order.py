"""Second-order wave loads in the batched solves (Model.analyzeCasesBatch / analyzeArrayBatch,
DesignBatch.solve): the batched counterpart of what Model.solveDynamics does per case.

The reference adds the difference-frequency force of a QTF to the excitation of a FOWT whose
platform sets potSecOrder (raft/raft_model.py:899-1083):
  potSecOrder == 2  the QTF comes from a WAMIT .12d file: the force of sea state 0 enters the
                    drag fixed point (F_lin, :903-904, :914), the force of every further sea
                    state enters that sea state's excitation (:1059-1061);
  potSecOrder == 1  the slender-body QTF is computed from the RAO of the first converged
                    response; the force then enters F_lin and the fixed point runs again from
                    iteration 1 with the un-relaxed XiLast (:966-989).  A further
                    sea state would index the QTF's one-heading axis with waveHeadInd > 0 and
                    raise IndexError (:1077, raft/raft_fowt.py:1442-1456).
Here the same sequence runs over a whole batch: one rh_sea_state launch for the spectra, one
rh_force_2nd_batch launch per FOWT for the file-QTF loads, the first pass of every case in one
rh_solve_cases launch, the slender-body QTF + force of each case that converged, and the
second pass of those cases in one more rh_solve_cases launch.  Each case gets the arithmetic
solveDynamics gives it (the same kernels on the same inputs).
"""
import numpy as np

from . import _native as N
from .hydro_math import DEG2RAD
from .solver import CaseSet, solve_batch


def order_of(owner):
    """potSecOrder of a view's FOWT (0 for host-only designs: they carry no QTF)."""
    return int(getattr(owner, "potSecOrder", 0) or 0)


def qtf_index_error(ih):
    """The reference's error for a slender-body QTF of sea state ih > 0."""
    return IndexError(f"index {ih} is out of bounds for axis 2 with size 1")


def sea_spectra(dd, cs_spectrum, Hs, Tp, gamma):
    """S and zeta [n, nw] of n sea states on design dd's grid (rh_sea_state, one launch)."""
    torch = dd.torch
    dev = dd.device
    n = len(Hs)
    f64 = dict(dtype=torch.float64, device=dev)
    S = torch.empty([n, dd.nw], **f64)
    zeta = torch.empty([n, dd.nw], **f64)
    if n == 0:
        return S, zeta
    spec = torch.tensor(np.asarray(cs_spectrum, dtype=np.int32), dtype=torch.int32, device=dev)
    H, T, G = (torch.tensor(np.asarray(x, dtype=float), **f64) for x in (Hs, Tp, gamma))
    N.check(N.lib().rh_sea_state(N.context(dd.dev_index), n, dd.nw, N.ptr(dd.w), float(dd.dw), N.ptr(spec), N.ptr(H),
                                 N.ptr(T), N.ptr(G), N.ptr(S), N.ptr(zeta), N.stream_handle(torch, dev)), "rh_sea_state")
    return S, zeta


QTF_CHUNK = 32     # QTFs of one stack in the potSecOrder = 1 second pass (15 MB each on the C3 grid)


def force_batch(dd, qdev, qtfs, qidx, S):
    """rh_force_2nd_batch: the 'qtf'-mode force of n sea states (calcHydroForce_2ndOrd,
    raft/raft_fowt.py:1788-1810).  qtfs: list of [n2, n2, 6] device QTFs on qdev's grid; qidx:
    per sea state, which one (or one [m, n2, n2, 6] tensor); S [n, nw].  Returns (f [n, 6, nw] complex, f_mean [n, 6])."""
    torch = dd.torch
    dev = dd.device
    n, nw = S.shape[0], dd.nw
    f = torch.empty([n, 6, nw], dtype=torch.complex128, device=dev)
    fm = torch.empty([n, 6], dtype=torch.float64, device=dev)
    if n == 0:
        return f, fm
    if torch.is_tensor(qtfs) and qtfs.dim() == 4:     # already one stack [m, n2, n2, 6]
        stack = qtfs.contiguous()
    else:
        stack = qtfs[0][None] if len(qtfs) == 1 else torch.stack(qtfs)
        stack = stack.contiguous()
    qi = torch.tensor(np.asarray(qidx, dtype=np.int32), dtype=torch.int32, device=dev)
    S = S.contiguous()
    N.check(N.lib().rh_force_2nd_batch(N.context(dd.dev_index), n, qdev.n2, N.ptr(qdev.w2), N.ptr(stack),
                                       int(stack.shape[0]), N.ptr(qi), nw, N.ptr(dd.w), float(dd.dw), N.ptr(S),
                                       N.ptr(f), N.ptr(fm), N.stream_handle(torch, dev)), "rh_force_2nd_batch")
    f._keep = (stack, qi, S)
    return f, fm


def file_qtf_forces(dd, fowt, betas, S):
    """Forces of the external (.12d) QTF of `fowt` for sea states with headings betas [rad]
    and spectra S [n, nw]: the QTF interpolated to each distinct heading once
    (FOWT._file_qtf_device, raft/raft_fowt.py:1752-1757), one batched force launch."""
    uniq = list(dict.fromkeys(float(b) for b in betas))
    ops = [fowt._file_qtf_device(b) for b in uniq]
    qdev = ops[0][0]
    where = {b: i for i, b in enumerate(uniq)}
    return force_batch(dd, qdev, [qt for _, qt in ops], [where[float(b)] for b in betas], S)


def solve_batch_2nd(views, owners, cs, nIter, XiStart, tol, want, prepared=None, F_wave=None, out=None):
    """solve_batch with the second-order loads of every case whose FOWT sets potSecOrder.
    views: DeviceDesign (or CaseMB) list; owners[v]: the FOWT whose potSecOrder, QTF and
    M_struc view v uses (None: first order only).  Adds to the result:
      iters_pair [n, 2]   drag solves of the first and second pass (0: no second pass; the
                          count of a potSecOrder=1 case is a pair)
      f2nd_mean  [n, 6]   mean drift of sea state 0 (Fhydro_2nd_mean[0])
      Fhydro_2nd [n, 6, nw] the force itself, when "Fhydro_2nd" is in want
    and iters / status / every output of the final pass.  Cases of first-order FOWTs are
    solved exactly as solve_batch solves them (out: solve_batch's preallocated outputs, first-order
    batches only)."""
    torch = views[0].torch
    dev = views[0].device
    n, nw = cs.n, views[0].nw
    vorder = np.array([order_of(o) for o in owners], dtype=np.int64)
    if not np.any(vorder > 0):
        return solve_batch(views, cs, nIter, XiStart, tol, want=want, prepared=prepared, F_wave=F_wave, out=out)
    order = vorder[cs.design_idx]
    if not np.any(order > 0):
        return solve_batch(views, cs, nIter, XiStart, tol, want=want, prepared=prepared, F_wave=F_wave, out=out)
    if out is not None:
        raise ValueError("solve_batch_2nd: preallocated outputs (out=) are for first-order batches")
    if F_wave is not None and np.any(order == 1):
        raise NotImplementedError("potSecOrder=1 in a coupled array: the reference adds the force to F_lin[i1:i2] "
                                  "of the whole system (raft/raft_model.py:988, SURVEY.md Q5)")
    S, _ = sea_spectra(views[0], cs.spectrum, cs.Hs, cs.Tp, cs.gamma)
    fext = torch.zeros([n, 6, nw], dtype=torch.complex128, device=dev)
    fmean = torch.zeros([n, 6], dtype=torch.float64, device=dev)
    # potSecOrder 2: the file QTF's force of sea state 0 inside the fixed point (:903-904)
    oid = np.array([id(o) for o in owners], dtype=object)
    for ow in {id(owners[int(v)]): owners[int(v)] for v in np.unique(cs.design_idx)}.values():
        if order_of(ow) != 2:
            continue
        sel = np.nonzero((order == 2) & (oid[cs.design_idx] == id(ow)))[0]
        st = torch.tensor(sel, dtype=torch.long, device=dev)
        f, fm = file_qtf_forces(views[int(cs.design_idx[sel[0]])], ow, cs.heading[sel] * DEG2RAD,
                                S.index_select(0, st))
        fext.index_copy_(0, st, f)
        fmean.index_copy_(0, st, fm)
    one = np.any(order == 1)
    want1 = tuple(want) + (("rao", "Xi_prev") if one else ())
    res = solve_batch(views, cs, nIter, XiStart, tol, want=want1, prepared=prepared, fext=fext, F_wave=F_wave)
    iters_pair = torch.zeros([n, 2], dtype=torch.int32, device=dev)
    iters_pair[:, 0] = res["iters"]
    if one:
        status = res["status"].cpu().numpy()
        sel = np.nonzero((order == 1) & (status == N.RH_CASE_CONVERGED))[0]
        if len(sel):
            _second_pass(views, owners, cs, sel, res, S, fext, fmean, nIter, XiStart, tol, want)
            st = torch.tensor(sel, dtype=torch.long, device=dev)
            iters_pair[st, 1] = res["iters"].index_select(0, st)
        for k in ("rao", "Xi_prev"):
            if k not in want:
                res.pop(k, None)
    res["iters_pair"] = iters_pair
    res["f2nd_mean"] = fmean
    if "Fhydro_2nd" in want:
        res["Fhydro_2nd"] = fext
    res._keep = (res._keep, fext, S)
    return res


def _second_pass(views, owners, cs, sel, res, S, fext, fmean, nIter, XiStart, tol, want):
    """potSecOrder=1 cases that converged: the slender-body QTF of each case's RAO
    (calcQTF_slenderBody(0, Xi0), raft/raft_model.py:978-981), its force with the case's
    spectrum (:987), and the fixed point again from iteration 1 with the un-relaxed XiLast
    (:973-988), all second passes in one launch; their outputs replace the first pass's."""
    torch = views[0].torch
    dev = views[0].device
    f64 = dict(dtype=torch.float64, device=dev)
    mass = {}
    # the converged cases grouped by QTF (design view, heading): each group's QTFs go into one
    # stack (chunks of QTF_CHUNK) and its forces come from one rh_force_2nd_batch launch; after
    # a QtfDevice's first QTF the incident-wave parts are kept (rh_qtf_slender_ext, the same bits)
    groups = {}
    for c in sel:
        v = int(cs.design_idx[c])
        groups.setdefault((v, float(cs.heading[c])), []).append(c)
    for (v, hdg), cases in groups.items():
        fowt, dd = owners[v], views[v]
        qd = fowt._qtf_device(hdg * DEG2RAD)
        if id(fowt) not in mass:
            mass[id(fowt)] = torch.tensor(np.asarray(fowt.M_struc, dtype=float), **f64).contiguous()
        for lo in range(0, len(cases), QTF_CHUNK):
            cc = cases[lo:lo + QTF_CHUNK]
            stack = torch.empty([len(cc), qd.n2, qd.n2, 6], dtype=torch.complex128, device=dev)
            for j, c in enumerate(cc):
                qd.qtf(dd.w, res["rao"][c].contiguous(), mass[id(fowt)], out=stack[j],
                       incident_cached=getattr(qd, "_incident_ready", False))
            idx = torch.tensor(cc, dtype=torch.long, device=dev)
            f, fm = force_batch(dd, qd, stack, np.arange(len(cc)), S.index_select(0, idx))
            fext.index_copy_(0, idx, f)
            fmean.index_copy_(0, idx, fm)   # (the stack is freed in stream order)
    st = torch.tensor(sel, dtype=torch.long, device=dev)
    sub = CaseSet(cs.design_idx[sel], cs.heading[sel], cs.spectrum[sel], cs.Hs[sel], cs.Tp[sel], cs.gamma[sel])
    fx = fext.index_select(0, st).contiguous()
    xi0 = res["Xi_prev"].index_select(0, st).contiguous()
    res2 = solve_batch(views, sub, nIter, XiStart, tol, want=tuple(want), fext=fx, Xi_init=xi0, first_iter=1)
    for k, v in res2.items():
        if k in res:
            res[k].index_copy_(0, st, v)
    res._keep = (res._keep, res2, fx, xi0)
