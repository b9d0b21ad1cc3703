"""Device tables for the slender-body QTF.

Per design, per second-order grid and heading: the static node/member/Kim-Yue tables of
include/rafthip.h (rh_qtf_design), built in librafthip on the host (rh_qtf_tables, from one
record per member: member_record) -- build_tables below states the same tables in NumPy and is
what tests/test_qtf_tables.py checks the native ones against.  The only host arithmetic is
geometry bookkeeping; the
Hankel-function table 0.5 (H1_{n-1}(kR) - H1_{n+1}(kR)) that the reference evaluates with
scipy.special.hankel1 (raft/raft_member.py:1104-1107) is built on the device
(rh_qtf_hankel), and every per-pair quantity is computed on the device by rh_qtf_slender.
"""
import ctypes

import numpy as np
from scipy.special import hankel1

from . import _native as N

QN_COUNT, QM_COUNT, KR_COUNT = 46, 36, 6


def hank_table(kk, R):
    """[n2, 12] table D_n(k R), n = 0..11 (orders -1..12 of scipy's hankel1): the host
    restatement rh_qtf_hankel is tested against (tests/test_gpu_qtf.py)."""
    x = np.asarray(kk, dtype=float) * R
    H = hankel1(np.arange(-1, 13)[:, None], x[None, :])         # [14, n2], one ufunc call
    D = 0.5 * (H[0:12] - H[2:14])                              # D_n = 0.5 (H_{n-1} - H_{n+1})
    return D.T.copy()


def build_tables(fowt, w2, k2, beta, host_hankel=False):
    """Static QTF tables of a FOWT for grid (w2, k2) and heading beta [rad].  The Hankel
    table is built on the host only with host_hankel=True (the device builds it otherwise).
    Each member's submerged nodes are tabulated with whole-array operations (the per-node
    arithmetic of raft/raft_fowt.py:1468-1502, 1532-1587 elementwise)."""
    rho, g, h = float(fowt.rho_water), float(fowt.g), float(fowt.depth)
    nblocks, mcols, kcols, hank = [], [], [], []
    qmstart, kstart = [0], [0]
    for mem in fowt.memberList:
        if mem.rA[2] > 0 and mem.rB[2] > 0:                     # entirely above water (:1461)
            continue
        circ = mem.shape == "circular"
        p1M, p2M, qM = mem.p1Mat, mem.p2Mat, mem.qMat
        sub = np.nonzero(mem.r[:, 2] < 0)[0]
        nsub = len(sub)
        last_cm = last_ca = np.zeros([3, 3])
        if nsub:
            ls = mem.ls[sub]
            Ca_p1, Ca_p2, Ca_End = (np.interp(ls, mem.stations, getattr(mem, k)) for k in ("Ca_p1", "Ca_p2", "Ca_End"))
            r = mem.r[sub]
            dls = mem.dls[sub]
            ds = np.asarray(mem.ds, dtype=float)[sub]
            drs = np.asarray(mem.drs, dtype=float)[sub]
            if circ:
                v_i = 0.25 * np.pi * ds ** 2 * dls
                ve = np.pi / 12.0 * np.abs((ds + drs) ** 3 - (ds - drs) ** 3)
            else:
                v_i = ds[:, 0] * ds[:, 1] * dls
                ve = np.pi / 12.0 * (np.mean(ds + drs, axis=1) ** 3 - np.mean(ds - drs, axis=1) ** 3)
            part = r[:, 2] + 0.5 * dls > 0                        # Q12
            v_i = np.where(part, v_i * (0.5 * dls - r[:, 2]) / np.where(part, dls, 1.0), v_i)
            CmM = (1. + Ca_p1)[:, None] * p1M.ravel() + (1. + Ca_p2)[:, None] * p2M.ravel()
            CaM = Ca_p1[:, None] * p1M.ravel() + Ca_p2[:, None] * p2M.ravel()
            last_cm, last_ca = CmM[-1].reshape(3, 3), CaM[-1].reshape(3, 3)
            blk = np.empty([nsub, QN_COUNT])
            blk[:, 0:3] = r
            blk[:, 3:6] = mem.q
            blk[:, 6] = v_i
            blk[:, 7] = ve
            blk[:, 8] = mem.a_i[sub]
            blk[:, 9] = Ca_End
            blk[:, 10:19] = CmM
            blk[:, 19:28] = CaM
            blk[:, 28:37] = (p1M + p2M).ravel()
            blk[:, 37:46] = qM.ravel()
            nblocks.append(blk)
        qmstart.append(qmstart[-1] + nsub)
        wl = mem.r[-1, 2] * mem.r[0, 2] < 0
        rint = np.zeros(3)
        awl = 0.0
        if wl:
            rint = mem.r[0] + (mem.r[-1] - mem.r[0]) * (0. - mem.r[0, 2]) / (mem.r[-1, 2] - mem.r[0, 2])
            i_wl = np.where(mem.r[:, 2] < 0)[0][-1]
            if circ:
                d_wl = 0.5 * (mem.ds[i_wl] + mem.ds[i_wl + 1]) if i_wl != len(mem.ds) - 1 else mem.ds[i_wl]
                awl = 0.25 * np.pi * d_wl ** 2
            else:
                if i_wl != len(mem.ds) - 1:
                    d1, d2 = 0.5 * (mem.ds[i_wl, 0] + mem.ds[i_wl + 1, 0]), 0.5 * (mem.ds[i_wl, 1] + mem.ds[i_wl + 1, 1])
                else:
                    d1, d2 = mem.ds[i_wl, 0], mem.ds[i_wl, 1]
                awl = d1 * d2
        # Kim & Yue (raft_member.py:1111-1200)
        kay = bool(mem.MCF) and (mem.rA[2] * mem.rB[2] < 0)
        pf = np.zeros(3)
        rwl = np.zeros(3)
        if kay:
            cb, sb = np.cos(beta), np.sin(beta)
            bv = np.array([cb, sb, 0])
            pf = np.dot(bv, mem.p1) * mem.p1 + np.dot(bv, mem.p2) * mem.p2
            pf = pf / np.linalg.norm(pf)
            rwl = mem.rA + (mem.rB - mem.rA) * (0 - mem.rA[2]) / (mem.rB[2] - mem.rA[2])
            R = np.interp(0, mem.r[:, 2], 0.5 * np.array(mem.ds))
            kcols.append([R, 0.0, 0.0, *rwl])
            if host_hankel:
                hank.append(hank_table(k2, R))
            ds_all = np.asarray(mem.ds, dtype=float)
            il = np.nonzero(mem.r[:-1, 2] <= 0)[0]                 # intervals whose first node is wet
            if len(il):
                z1 = mem.r[il, 2]
                z2 = np.where(mem.r[il + 1, 2] > 0, 0.0, mem.r[il + 1, 2])
                R1 = np.where(mem.dls[il] == 0, ds_all[il], ds_all[il] / 2)
                R2 = np.where(mem.dls[il + 1] == 0, ds_all[il], ds_all[il + 1] / 2)   # Q9
                Rm = 0.5 * (R1 + R2)
                mid = 0.5 * (mem.r[il] + mem.r[il + 1])
                for j in range(len(il)):
                    kcols.append([Rm[j], z1[j], z2[j], *mid[j]])
                    if host_hankel:
                        hank.append(hank_table(k2, Rm[j]))
        kstart.append(len(kcols))
        mcols.append([1.0 if wl else 0.0, *rint, awl, *last_cm.ravel(), *last_ca.ravel(), *mem.p1, *mem.p2,
                      1.0 if kay else 0.0, *pf, *rwl])
    qnode = np.concatenate(nblocks).T.copy() if nblocks else np.zeros([QN_COUNT, 0])
    qmemb = np.array(mcols, dtype=float).T.copy() if mcols else np.zeros([QM_COUNT, 0])
    kray = np.array(kcols, dtype=float).T.copy() if kcols else np.zeros([KR_COUNT, 0])
    hk = np.array(hank, dtype=complex) if hank else None
    assert qnode.shape[0] == QN_COUNT and qmemb.shape[0] == QM_COUNT
    return dict(qnode=qnode, qmemb=qmemb, kray=kray, hank=hk, qmstart=np.array(qmstart, dtype=np.int32),
                kstart=np.array(kstart, dtype=np.int32), rho=rho, g=g, h=h)


def member_record(mem):
    """One member's record for rh_qtf_tables (format: csrc/rh_qtf_host.h)."""
    return np.concatenate(((1.0 if mem.shape == "circular" else 0.0, 1.0 if mem.MCF else 0.0, len(mem.r),
                            len(mem.stations)), mem.rA, mem.rB, mem.p1, mem.p2, mem.q, mem.p1Mat, mem.p2Mat, mem.qMat,
                           mem.r, mem.ls, mem.dls, mem.ds, mem.drs, mem.a_i, mem.stations, mem.Ca_p1, mem.Ca_p2,
                           mem.Ca_End), axis=None)


def table_capacity(fowt):
    """Doubles that native_tables may need for a FOWT's tables and index tables (an upper
    bound: every node submerged and a Kim & Yue row per node)."""
    mems = fowt.memberList
    return (QN_COUNT + KR_COUNT) * sum(len(m.r) for m in mems) + QM_COUNT * len(mems) + len(mems) + 1


def native_tables(fowt, beta, buf=None, off=0):
    """rh_qtf_tables: the tables of build_tables (without the Hankel table), written into
    buf[off:] (float64; allocated when None) as qnode | qmemb | kray back to back, followed by
    qmstart | kstart as int32 bytes.  Returns (buf, end, dict of numpy views like build_tables)."""
    mems = fowt.memberList
    rec = np.concatenate([member_record(m) for m in mems]) if mems else np.zeros(0)
    capi = 2 * (len(mems) + 1)
    cap = table_capacity(fowt) - capi // 2
    need = off + cap + capi // 2
    if buf is None:
        buf = np.empty(need)
    elif buf.size < need:
        raise ValueError("native_tables: buffer too small")
    iout = np.empty(capi, dtype=np.int32)
    cnt = np.zeros(3, dtype=np.int32)
    tab = buf[off:]
    N.check(N.lib().rh_qtf_tables(len(mems), rec.ctypes.data, rec.size, float(beta), tab.ctypes.data, cap,
                                  iout.ctypes.data, capi, cnt.ctypes.data), "rh_qtf_tables")
    nq, nmq, nkr = (int(x) for x in cnt)
    o1, o2, o3 = QN_COUNT * nq, QN_COUNT * nq + QM_COUNT * nmq, QN_COUNT * nq + QM_COUNT * nmq + KR_COUNT * nkr
    ni = 2 * (nmq + 1)
    ints = tab[o3:o3 + (ni + 1) // 2].view(np.int32)[:ni]
    ints[:] = iout[:ni]
    t = dict(qnode=tab[:o1].reshape(QN_COUNT, nq), qmemb=tab[o1:o2].reshape(QM_COUNT, nmq),
             kray=tab[o2:o3].reshape(KR_COUNT, nkr), hank=None, qmstart=ints[:nmq + 1], kstart=ints[nmq + 1:],
             rho=float(fowt.rho_water), g=float(fowt.g), h=float(fowt.depth))
    return buf, off + o3 + (ni + 1) // 2, t


_STAGING = {}


def _staging(torch, dev, n):
    """A pinned host buffer of >= n doubles per device, reused: the tables of a new QtfDevice are
    written there natively and go up in one asynchronous copy.  Waits for the previous copy out
    of it first."""
    st = _STAGING.get(dev.index)
    if st is not None:
        st[1].synchronize()
    if st is None or st[0].numel() < n:
        st = [torch.empty(max(n, 8192), dtype=torch.float64, pin_memory=True), torch.cuda.Event()]
        _STAGING[dev.index] = st
    return st


class QtfDevice:
    """Device copy of the QTF tables + workspace for one (design, grid, heading)."""

    def __init__(self, fowt, w2, k2, beta, device):
        import torch
        self.torch = torch
        self.dev = torch.device("cuda", device)
        self.dev_index = device
        self.n2 = n2 = len(w2)
        self.beta = float(beta)
        # the grid, the three tables and the two index tables, written natively into one pinned
        # buffer, in one asynchronous upload
        stage = _staging(torch, self.dev, 2 * n2 + table_capacity(fowt))
        host = stage[0].numpy()
        host[:n2] = w2
        host[n2:2 * n2] = k2
        _, end, t = native_tables(fowt, beta, host, 2 * n2)
        dev_flat = stage[0][:end].to(self.dev, non_blocking=True)
        stage[1].record(torch.cuda.current_stream(self.dev))
        self.host = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in t.items()}
        self.nq, self.nmq, self.nkr = t["qnode"].shape[1], t["qmemb"].shape[1], t["kray"].shape[1]
        self.w2, self.k2 = dev_flat[:n2], dev_flat[n2:2 * n2]
        off = 2 * n2
        views = []
        for rows, n in ((QN_COUNT, self.nq), (QM_COUNT, self.nmq), (KR_COUNT, self.nkr)):
            views.append(dev_flat[off:off + rows * n].view(rows, n))
            off += rows * n
        self.qnode, self.qmemb, self.kray = views
        ni = 2 * (self.nmq + 1)
        ints = dev_flat[off:off + (ni + 1) // 2].view(torch.int32)[:ni]
        self.qmstart, self.kstart = ints[:self.nmq + 1], ints[self.nmq + 1:]
        # Kim & Yue Hankel table [nkr][n2][12], built on the device from k2 and the radii
        self.hank = (torch.empty if self.nkr else torch.zeros)([max(self.nkr, 1), self.n2, 12], dtype=torch.complex128,
                                                               device=self.dev)
        if self.nkr:
            N.check(N.lib().rh_qtf_hankel(N.context(device), self.n2, N.ptr(self.k2), self.nkr, N.ptr(self.kray),
                                          N.ptr(self.hank), N.stream_handle(torch, self.dev)), "rh_qtf_hankel")
        self.rho, self.g, self.h = t["rho"], t["g"], t["h"]
        # the MFMA pair path needs the upper triangle to be i2 >= i1 and nk = k2 - k1
        w2a, k2a = np.asarray(w2, dtype=float), np.asarray(k2, dtype=float)
        self.order = int(bool(np.all(np.diff(w2a) > 0) and np.all(np.diff(k2a) > 0)))
        self.struct_ = self.struct()
        nbytes = N.lib().rh_qtf_workspace_bytes(ctypes.byref(self.struct_))
        self.work = torch.empty(int(nbytes) // 16 + 1, dtype=torch.complex128, device=self.dev)
        self.work_bytes = int(self.work.numel() * 16)

    def struct(self):
        q = N.RhQtfDesign()
        q.n2, q.nq, q.nmq, q.nkr = self.n2, self.nq, self.nmq, self.nkr
        q.beta, q.depth, q.rho, q.g = self.beta, self.h, self.rho, self.g
        q.w2, q.k2 = N.ptr(self.w2), N.ptr(self.k2)
        q.qnode, q.qmemb, q.qmstart, q.kstart = N.ptr(self.qnode), N.ptr(self.qmemb), N.ptr(self.qmstart), N.ptr(self.kstart)
        q.kray, q.hank = N.ptr(self.kray), N.ptr(self.hank)
        q.order = self.order
        return q

    def qtf(self, w, Xi0, M66, out=None, group=None, on_computed=None, incident_cached=False):
        """Run rh_qtf_slender: w [nw] / Xi0 [6, nw] device tensors -> qtf [n2, n2, 6] device tensor.
        Sharding is opt-in: only with an explicit process `group` of world > 1 are the pairs
        row-sharded over its ranks (raft/parallel.py) -- a collective every rank of the group
        must enter with the same inputs -- and every rank returns the full matrix.  group=None
        (what FOWT.calcQTF_slenderBody passes) never communicates, so ranks that each solve
        their own cases or designs can call it independently.  on_computed: optional callback
        run after this rank's pair kernels are enqueued, before any exchange (bench timing).
        incident_cached: this QtfDevice's workspace holds the incident-wave parts of an earlier
        whole-QTF call on the default (MFMA) path, on this stream or one synchronised with it
        (rh_qtf_slender_ext RH_QTF_INCIDENT_CACHED): only the RAO-dependent parts run; the same
        bits as a full call."""
        torch = self.torch
        from .parallel import assemble_qtf, world_of
        if group is not None and world_of(group)[1] > 1:
            return assemble_qtf(lambda o, r, n: self.qtf_rows(w, Xi0, M66, o, r, n), self.hermitian_fill, self.n2,
                                device=self.dev, group=group, on_computed=on_computed)
        if incident_cached and not getattr(self, "_incident_ready", False):
            raise ValueError("QtfDevice.qtf: incident_cached needs an earlier whole-QTF call on this device")
        if out is None:
            out = torch.empty([self.n2, self.n2, 6], dtype=torch.complex128, device=self.dev)
        N.check(N.lib().rh_qtf_slender_ext(N.context(self.dev_index), ctypes.byref(self.struct_), int(w.numel()),
                                           N.ptr(w), N.ptr(Xi0), N.ptr(M66), N.ptr(out), N.ptr(self.work),
                                           ctypes.c_longlong(self.work_bytes),
                                           N.RH_QTF_INCIDENT_CACHED if incident_cached else 0,
                                           N.stream_handle(torch, self.dev)),
                "rh_qtf_slender_ext")
        self._incident_ready = True
        if on_computed is not None:
            on_computed()
        return out


    def qtf_rows(self, w, Xi0, M66, out, rank, nrank):
        """rh_qtf_slender_rows: the upper-triangle pair tiles of `rank` (parallel.qtf_tiles) into `out`."""
        N.check(N.lib().rh_qtf_slender_rows(N.context(self.dev_index), ctypes.byref(self.struct_), int(w.numel()),
                                            N.ptr(w), N.ptr(Xi0), N.ptr(M66), int(rank), int(nrank), N.ptr(out),
                                            N.ptr(self.work), ctypes.c_longlong(self.work_bytes),
                                            N.stream_handle(self.torch, self.dev)), "rh_qtf_slender_rows")
        return out

    def hermitian_fill(self, out):
        N.check(N.lib().rh_qtf_hermitian_fill(N.context(self.dev_index), self.n2, N.ptr(out),
                                              N.stream_handle(self.torch, self.dev)), "rh_qtf_hermitian_fill")
        return out


def force_2nd(qdev, qtf, w, dw, S0):
    """rh_force_2nd: (f_mean [6], f [6, nw]) device tensors."""
    torch = qdev.torch
    nw = int(w.numel())
    f = torch.empty([6, nw], dtype=torch.float64, device=qdev.dev)
    fm = torch.empty([6], dtype=torch.float64, device=qdev.dev)
    N.check(N.lib().rh_force_2nd(N.context(qdev.dev_index), qdev.n2, N.ptr(qdev.w2), N.ptr(qtf), nw, N.ptr(w),
                                 float(dw), N.ptr(S0), N.ptr(f), N.ptr(fm), N.stream_handle(torch, qdev.dev)),
            "rh_force_2nd")
    return fm, f


def force_2nd_spectrum(qdev, qtf, w, dw, S0):
    """rh_force_2nd_spectrum ('spectrum' mode, raft/raft_fowt.py:1760-1784): (f_mean [6],
    f [6, nw] complex with zero imaginary part, as the reference returns it) device tensors."""
    torch = qdev.torch
    nw = int(w.numel())
    f = torch.empty([6, nw], dtype=torch.float64, device=qdev.dev)
    fm = torch.empty([6], dtype=torch.float64, device=qdev.dev)
    Sf = torch.empty([6, qdev.n2], dtype=torch.float64, device=qdev.dev)
    N.check(N.lib().rh_force_2nd_spectrum(N.context(qdev.dev_index), qdev.n2, N.ptr(qdev.w2), N.ptr(qtf), nw,
                                          N.ptr(w), float(dw), N.ptr(S0), N.ptr(Sf), N.ptr(f), N.ptr(fm),
                                          N.stream_handle(torch, qdev.dev)), "rh_force_2nd_spectrum")
    return fm, torch.complex(f, torch.zeros_like(f))
