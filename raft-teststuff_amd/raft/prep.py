"""Per-design device tables: the host -> HBM layout of everything the kernels read.

Layout in HBM (one design, nn submerged nodes, nw bins, nh headings):
  node      float64 [RH_NF_COUNT][nn]     struct-of-arrays node table (wave-uniform reads)
  imat_mcf  complex128 [nn][9][nw]        only when some member uses MacCamy-Fuchs
  uhat      complex128 [nh][nn][3][nw]    unit-amplitude wave velocity, bins contiguous
  finer     complex128 [nh][6][nw]        unit-amplitude inertial excitation
  M, B      float64 [36] or [nw][36]      M_lin, B_lin (raft/raft_model.py:911-912)
  C         float64 [36]                  C_lin (raft/raft_model.py:913)
uhat is what the case kernel streams twice per drag iteration; bins are contiguous so a
wavefront (64 consecutive bins) reads 1 KiB per component per node.
"""
import ctypes

import numpy as np

from . import _native as N

SQRT_8_PI_NOTE = "Borgman factor sqrt(8/pi) applied on the device (raft/raft_fowt.py:1223)"


_TORCH = []


def _torch():
    if _TORCH:                # checked once per process (a DeviceDesign per design of a sweep block)
        return _TORCH[0]
    import torch
    if not torch.cuda.is_available():
        raise N.NativeError("librafthip needs a visible MI355X (torch.cuda.is_available() is False); "
                            "there is no CPU fallback")
    _TORCH.append(torch)
    return torch


def node_table(fowt):
    """Gather the submerged strip nodes of all members (reference member/node order) into
    the [RH_NF_COUNT][nn] table and the optional MCF Imat block.  Areas follow
    raft/raft_fowt.py:1199-1238 (incl. SURVEY.md Q4 for the rectangular axial area)."""
    cols = []
    mcf_blocks = []
    any_mcf = False
    mcols, mstart = [], [0]
    for mem in fowt.memberList:
        circ = mem.shape == "circular"
        nsub = int(np.sum(mem.r[:, 2] < 0))
        if nsub:
            rA = mem.rA - fowt.r6[:3]
            q, p1, p2 = mem.q, mem.p1, mem.p2
            mcols.append([*q, *np.cross(rA, q), *p1, *np.cross(rA, p1), *p2, *np.cross(rA, p2),
                          q @ q, p1 @ p1, p2 @ p2])
            mstart.append(mstart[-1] + nsub)
        for il in range(mem.ns):
            if not (mem.r[il, 2] < 0):
                continue
            ds, drs, dls = np.atleast_1d(mem.ds[il]), np.atleast_1d(mem.drs[il]), mem.dls[il]
            if circ:
                a_q = np.pi * ds[0] * dls
                a_p1 = ds[0] * dls
                a_p2 = ds[0] * dls
                a_end = np.abs(np.pi * ds[0] * drs[0])
            else:
                a_q = 2 * (ds[0] + ds[0]) * dls
                a_p1 = ds[0] * dls
                a_p2 = ds[1] * dls
                a_end = np.abs((ds[0] + drs[0]) * (ds[1] + drs[1]) - (ds[0] - drs[0]) * (ds[1] - drs[1]))
            r = mem.r[il]
            rr = mem.r[il] - fowt.r6[:3]
            use_mcf = bool(mem.MCF and mem.Imat_MCF is not None)
            any_mcf |= use_mcf
            col = [r[0], r[1], r[2], rr[0], rr[1], rr[2], *mem.q, *mem.p1, *mem.p2,
                   a_q, a_p1, a_p2, a_end,
                   mem.coef("Cd_q", il), mem.coef("Cd_p1", il), mem.coef("Cd_p2", il), mem.coef("Cd_End", il),
                   1.0 if circ else 0.0, mem.a_i[il], 1.0 if use_mcf else 0.0, *mem.Imat[il].ravel(),
                   mem.ls[il]]
            cols.append(col)
            mcf_blocks.append(mem.Imat_MCF[il].reshape(9, -1) if use_mcf else None)
    table = np.array(cols, dtype=float).T.copy() if cols else np.zeros([N.NF_COUNT, 0])
    members = np.array(mcols, dtype=float).T.copy() if mcols else np.zeros([N.MF_COUNT, 0])
    imat = None
    if any_mcf:
        imat = np.zeros([len(cols), 9, fowt.nw], dtype=complex)
        for i, blk in enumerate(mcf_blocks):
            if blk is not None:
                imat[i] = blk
    return table, imat, members, np.array(mstart, dtype=np.int32)


def linear_matrices(fowt):
    """M_lin, B_lin, C_lin without rotor aero (raft/raft_model.py:911-913).  Returns
    (M, B, C, per_bin) with M, B of shape [nw,6,6] when frequency dependent else [6,6]."""
    A_BEM = np.asarray(fowt.A_BEM)
    B_BEM = np.asarray(fowt.B_BEM)
    B_gyro = np.sum(fowt.B_gyro, axis=2) if getattr(fowt, "B_gyro", None) is not None and np.ndim(fowt.B_gyro) == 3 \
        else np.zeros([6, 6])
    per_bin = bool(np.any(A_BEM) or np.any(B_BEM))
    C = (fowt.C_struc + fowt.C_moor) + fowt.C_hydro
    A_aero, B_aero = getattr(fowt, "A_aero", None), getattr(fowt, "B_aero", None)
    if A_aero is not None and np.ndim(A_aero) == 4 and (np.any(A_aero) or np.any(B_aero)):
        # operating rotors: the reference's sums, in its order (raft/raft_model.py:887-889, 911-912)
        M_turb, B_turb = np.sum(A_aero, axis=3), np.sum(B_aero, axis=3)
        M = ((M_turb + fowt.M_struc[:, :, None]) + A_BEM) + fowt.A_hydro_morison[:, :, None]
        B = ((B_turb + fowt.B_struc[:, :, None]) + B_BEM) + B_gyro[:, :, None]
        return np.moveaxis(M, 2, 0).copy(), np.moveaxis(B, 2, 0).copy(), C, True
    if per_bin:
        M = (fowt.M_struc[:, :, None] + A_BEM) + fowt.A_hydro_morison[:, :, None]
        B = (fowt.B_struc[:, :, None] + B_BEM) + B_gyro[:, :, None]
        return np.moveaxis(M, 2, 0).copy(), np.moveaxis(B, 2, 0).copy(), C, True
    M = fowt.M_struc + fowt.A_hydro_morison
    B = fowt.B_struc + B_gyro
    return M, B, C, False


def host_tables(fowt):
    """Everything DeviceDesign uploads, computed on the host (NumPy only, so it can run in
    a host worker next to the rest of the per-design preparation): the real-valued tables
    packed into ONE float64 array (one host->device copy per design) plus their layout."""
    table, imat, members, mstart = node_table(fowt)
    nn, nm = table.shape[1], members.shape[1]
    M, B, C, per_bin = linear_matrices(fowt)
    parts = [("w", np.asarray(fowt.w, dtype=float)), ("k", np.asarray(fowt.k, dtype=float)),
             ("node", table if nn else np.zeros([N.NF_COUNT, 1])), ("memb", members if nm else np.zeros([N.MF_COUNT, 1])),
             ("M", np.asarray(M, dtype=float)), ("B", np.asarray(B, dtype=float)), ("C", np.asarray(C, dtype=float))]
    layout, off = {}, 0
    for name, a in parts:
        layout[name] = (off, a.shape)
        off += a.size
    packed = np.concatenate([np.ascontiguousarray(a).ravel() for _, a in parts])
    return dict(packed=packed, layout=layout, imat=imat, mstart=mstart, nn=nn, nm=nm, per_bin=per_bin)


class DeviceDesign:
    """Device-resident tables of one FOWT design (caller-owned torch buffers)."""

    def __init__(self, fowt, device=0, packed=None, mstart=None):
        """packed / mstart: this design's slices of device arrays the caller already holds
        (DesignBatch uploads every design's tables in one copy); otherwise uploaded here."""
        torch = _torch()
        self.torch = torch
        self.device = torch.device("cuda", device)
        self.dev_index = device
        self.nw = fowt.nw
        h = fowt.host_tables() if hasattr(fowt, "host_tables") else host_tables(fowt)
        self.nn, self.nm, self.per_bin = h["nn"], h["nm"], h["per_bin"]
        if packed is not None and packed.numel() != h["packed"].size:
            raise ValueError("DeviceDesign: packed slice does not match the design's tables")
        self._packed = packed if packed is not None else torch.tensor(h["packed"], dtype=torch.float64,
                                                                        device=self.device)
        # w, k, node, memb, M, B, C: contiguous views of the one upload, made on first use
        # (__getattr__); the descriptor takes their addresses from the layout directly
        self._layout = h["layout"]
        imat = h["imat"]
        self.imat = torch.tensor(imat, dtype=torch.complex128, device=self.device) if imat is not None else None
        self.mstart = mstart if mstart is not None else torch.tensor(h["mstart"], dtype=torch.int32, device=self.device)
        self.dw, self.depth, self.rho, self.g = float(fowt.dw), float(fowt.depth), float(fowt.rho_water), float(fowt.g)
        self.headings = None           # tuple of tabulated headings (rad)
        self.uhat = None
        self.finer = None
        self.kproj = None

    _TABLES = ("uhat", "kproj", "finer")

    def __getattr__(self, name):
        tab = self.__dict__.get("_tab")
        if tab is not None and name in self._TABLES:     # a view of the batch's shared tables, made on first use
            v = self._tab_view(name)
            self.__dict__[name] = v
            return v
        lay = self.__dict__.get("_layout")
        if lay is None or name not in lay:
            raise AttributeError(name)
        off, shape = lay[name]
        v = self._packed[off:off + int(np.prod(shape))].view(*shape)
        self.__dict__[name] = v
        return v

    def _tab_view(self, name):
        base, off, shape = self._tab[name]
        return base[off:off + int(np.prod(shape))].view(*shape)

    def set_tables(self, tab, headings):
        """Point the wave tables at slices of shared allocations without making the views:
        tab[name] = (flat complex128 tensor, element offset, shape) for uhat, kproj, finer
        (raft/prep.py tabulate_batch; the views appear on first access)."""
        for name in self._TABLES:
            self.__dict__.pop(name, None)
        self._tab = tab
        self.headings = tuple(headings)
        self._tabver = getattr(self, "_tabver", 0) + 1

    def _tab_ptr(self, name):
        if name not in self.__dict__ and self.__dict__.get("_tab") is not None:
            base, off, _ = self._tab[name]
            return ctypes.c_void_p(base.data_ptr() + 16 * off)
        return N.ptr(self.__dict__.get(name))

    def _addr(self, name):
        return ctypes.c_void_p(self._packed.data_ptr() + 8 * self._layout[name][0])

    def struct(self):
        """The rh_design descriptor of the current tables (cached until they change)."""
        st = self.__dict__.get("_struct")
        key = (self.__dict__.get("_tabver", 0), self.__dict__.get("kproj"), self.headings)
        if st is not None and st[0][0] == key[0] and st[0][1] is key[1] and st[0][2] == key[2]:
            return st[1]
        d = self._make_struct()
        self._struct = (key, d)
        return d

    def _make_struct(self):
        d = N.RhDesign()
        d.nw, d.nn = self.nw, self.nn
        d.nhead = 0 if self.headings is None else len(self.headings)
        d.mb_per_bin = 1 if self.per_bin else 0
        d.dw, d.depth, d.rho, d.g = self.dw, self.depth, self.rho, self.g
        d.pdyn_rho_g = 1025.0 * 9.81   # getWaveKin defaults (raft/helpers.py:105, raft/raft_fowt.py:1109)
        d.w, d.k, d.node = self._addr("w"), self._addr("k"), self._addr("node")
        d.nm, d.memb, d.mstart = self.nm, self._addr("memb"), N.ptr(self.mstart)
        d.imat_mcf = N.ptr(self.imat)
        d.uhat, d.finer, d.kproj = self._tab_ptr("uhat"), self._tab_ptr("finer"), self._tab_ptr("kproj")
        d.M, d.B, d.C = self._addr("M"), self._addr("B"), self._addr("C")
        return d

    def ensure_headings(self, betas):
        """Tabulate unit-amplitude kinematics for the given headings (rad).  Returns the
        table index of each requested heading."""
        betas = [float(b) for b in np.atleast_1d(betas)]
        have = list(self.headings) if self.headings is not None else []
        missing = [b for b in dict.fromkeys(betas) if b not in have]
        if missing or self.uhat is None:
            allh = have + missing
            torch = self.torch
            nh = len(allh)
            self._tab = None
            self.uhat = torch.empty([nh, max(self.nn, 1), 3, self.nw], dtype=torch.complex128, device=self.device)
            self.finer = torch.empty([nh, 6, self.nw], dtype=torch.complex128, device=self.device)
            self.kproj = torch.empty([nh, max(self.nn, 1), 3, self.nw], dtype=torch.complex128, device=self.device)
            self.headings = tuple(allh)
            self._tabver = getattr(self, "_tabver", 0) + 1
            beta_t = torch.tensor(allh, dtype=torch.float64, device=self.device)
            d = self.struct()
            N.check(N.lib().rh_wave_tables(N.context(self.dev_index), ctypes.byref(d), N.ptr(beta_t),
                                           N.ptr(self.uhat), N.ptr(self.finer), N.ptr(self.kproj),
                                           N.stream_handle(torch, self.device)),
                    "rh_wave_tables")
            self._beta_keep = beta_t
        return [self.headings.index(b) for b in betas]

    def retabulate(self, stream=None):
        """Recompute the wave tables of the tabulated headings in place (same buffers, one
        rh_wave_tables launch): the per-design table work of a batch, e.g. inside a timed
        step.  The values are identical to the first tabulation."""
        if self.uhat is None:
            raise RuntimeError("retabulate: no headings tabulated yet (ensure_headings)")
        d = self.struct()
        s = stream if stream is not None else N.stream_handle(self.torch, self.device)
        N.check(N.lib().rh_wave_tables(N.context(self.dev_index), ctypes.byref(d), N.ptr(self._beta_keep),
                                       N.ptr(self.uhat), N.ptr(self.finer), N.ptr(self.kproj), s), "rh_wave_tables")


def descriptor_block(designs):
    """The rh_design descriptors of many designs as one ctypes array, filled column-wise in a
    numpy record array of rh_design's layout (DeviceDesign._make_struct's values, without a
    ctypes field write per field and design); each design's descriptor cache is set from it."""
    rec = np.zeros(len(designs), dtype=np.dtype(N.RhDesign))
    cols = {k: [] for k in rec.dtype.names}
    for d in designs:
        base = d._packed.data_ptr()
        lay = d._layout
        for k in ("w", "k", "node", "memb", "M", "B", "C"):
            cols[k].append(base + 8 * lay[k][0])
        for k in ("uhat", "finer", "kproj"):
            cols[k].append(d._tab_ptr(k).value or 0)
        cols["mstart"].append(d.mstart.data_ptr())
        cols["imat_mcf"].append(d.imat.data_ptr() if d.imat is not None else 0)
        cols["nw"].append(d.nw)
        cols["nn"].append(d.nn)
        cols["nm"].append(d.nm)
        cols["nhead"].append(0 if d.headings is None else len(d.headings))
        cols["mb_per_bin"].append(1 if d.per_bin else 0)
        cols["dw"].append(d.dw)
        cols["depth"].append(d.depth)
        cols["rho"].append(d.rho)
        cols["g"].append(d.g)
    cols["pdyn_rho_g"] = [1025.0 * 9.81] * len(designs)   # getWaveKin defaults (see _make_struct)
    for k, v in cols.items():
        rec[k] = v
    arr = (N.RhDesign * len(designs)).from_buffer(rec)
    arr._rec = rec                                         # (the array's memory)
    for j, d in enumerate(designs):
        d._struct = ((d.__dict__.get("_tabver", 0), d.__dict__.get("kproj"), d.headings), N.RhDesign.from_buffer_copy(arr[j]))
    return arr


def tabulate_batch(designs, design_idx, betas, launch_stream=None):
    """Wave tables of every (design, heading) pair a batch needs, in ONE rh_wave_tables_batch
    launch, for designs that have none yet (a fresh design sweep).  Returns the heading
    index of every case in its design's tables.  Tables of all designs share three device
    allocations; each DeviceDesign holds views.  launch_stream: run the launch there (after
    this stream's uploads, through an event) instead of on the current stream."""
    from .sweep_block import table_plan
    torch = designs[0].torch
    dev = designs[0].device
    head, di, nh, hstride, bm = table_plan(design_idx, betas)
    sel = [designs[int(i)] for i in di]
    nw = sel[0].nw
    rows = [int(k) * max(d.nn, 1) * 3 * nw for d, k in zip(sel, nh)]
    c128 = dict(dtype=torch.complex128, device=dev)
    U = torch.empty([sum(rows)], **c128)
    K = torch.empty([sum(rows)], **c128)
    Fi = torch.empty([int(nh.sum()) * 6 * nw], **c128)
    ou = of = 0
    for j, (d, k) in enumerate(zip(sel, nh)):
        k = int(k)
        hs = bm[j, :k]
        shp = (k, max(d.nn, 1), 3, nw)
        d.set_tables({"uhat": (U, ou, shp), "kproj": (K, ou, shp), "finer": (Fi, of, (k, 6, nw))},
                     [float(b) for b in hs])
        ou, of = ou + rows[j], of + k * 6 * nw
    beta_t = torch.tensor(bm, dtype=torch.float64, device=dev)
    for j, d in enumerate(sel):
        d._beta_keep = beta_t[j, :int(nh[j])]
    arr = descriptor_block(sel)
    if launch_stream is not None:
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
        launch_stream.wait_event(ev)
        s = ctypes.c_void_p(launch_stream.cuda_stream)
    else:
        s = N.stream_handle(torch, dev)
    N.check(N.lib().rh_wave_tables_batch(N.context(sel[0].dev_index), arr, len(sel), N.ptr(beta_t), hstride, s),
            "rh_wave_tables_batch")
    return head
