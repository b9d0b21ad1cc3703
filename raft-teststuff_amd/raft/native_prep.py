"""Native per-design host preparation (rh_prep_designs, csrc/rh_prep.h): the design sweep's
host path without per-design interpreter work.

A design dict is flattened into one float64 spec record (design_spec: the parsed member,
rotor and statics inputs, with the reference's input rules of raft/member.py and
raft/hydro_math.get_from_dict); librafthip then builds members, statics, added mass and the
device tables of every design on host threads (the work of Model/FOWT setup,
raft/raft_model.py:30-170, raft/raft_fowt.py:291-565, 848-880, that raft/batch.py
prepare_design does in Python).  The Python path stays the parity reference
(tests/test_native_prep.py compares every table and matrix).
"""
import ctypes

import numpy as np

from . import _native as N
from .hydro_math import get_from_dict

MAGIC = 7301
STATIC_KEYS = ("M_struc", "B_struc", "C_struc", "C_hydro", "C_moor")


def _vec(d, key, n, default=None, index=None):
    """get_from_dict(d, key, shape=n, default=default, index=index) as a list of n floats
    (raft/hydro_math.py get_from_dict: scalars are tiled; with `index`, a 1-D list gives its
    index-th entry tiled and a 2-D list its index-th column)."""
    if key not in d:
        if default is None:
            raise ValueError(f"Key '{key}' not found in input file...")
        return [float(default)] * n
    val = d[key]
    if not isinstance(val, (list, tuple, np.ndarray)):
        return [float(val)] * n
    if len(val) != n:
        raise ValueError(f"Value for key '{key}' is not the expected size of {n} and is instead: {val}")
    if index is None:
        return [float(v) for v in val]
    if not isinstance(val[0], (list, tuple, np.ndarray)):
        if 0 <= index < len(val):
            return [float(val[index])] * n
        raise ValueError(f"Value for index '{index}' is not within the size of {val} (len={len(val)})")
    return [float(v[index]) for v in val]


def _pairs(d, key, n):
    """get_from_dict(d, key, shape=[n, 2]) flattened (rectangular side lengths)."""
    val = d[key]
    if not isinstance(val, (list, tuple, np.ndarray)):
        return [float(val)] * (2 * n)
    a = np.asarray(val, dtype=float)
    if a.shape == (n, 2):
        return a.ravel().tolist()
    if a.ndim == 1 and len(a) == 2:
        return a.tolist() * n
    raise ValueError(f"Value for key '{key}' is not a compatible size for target size of {[n, 2]} and is instead: {val}")


def _scalar(d, key, default):
    if key not in d:
        return default
    val = d[key]
    if isinstance(val, (list, tuple, np.ndarray)):
        raise ValueError(f"Value for key '{key}' is expected to be a scalar but instead is: {val}")
    return val


def _member_spec(mi, heads, dlsMax_default, potModMaster, is_platform):
    """One reference member entry (all its heading copies) as a list of spec values; the
    parsing of raft/member.py Member.__init__ (raft/raft_member.py:23-96)."""
    potMod = bool(_scalar(mi, "potMod", False))
    dls = mi.get("dlsMax")
    if is_platform:
        if potModMaster in [1]:
            potMod = False
        elif potModMaster in [2, 3]:
            potMod = True
        if dls is None:
            dls = dlsMax_default
    dlsMax = 5.0 if dls is None else float(np.atleast_1d(dls)[0])
    st = [float(x) for x in mi["stations"]]
    n = len(st)
    if n < 2:
        raise ValueError("At least two stations entries must be provided")
    if sorted(st) != st:
        raise ValueError(f"Member {mi['name']}: the station list is not in ascending order.")
    shape = str(mi["shape"])[0].lower()
    if shape not in ("c", "r"):
        raise ValueError("The only allowable shape strings are circular and rectangular")
    circ = shape == "c"
    mcf = bool(_scalar(mi, "MCF", False)) and circ
    dd = _vec(mi, "d", n) if circ else _pairs(mi, "d", n)
    has_t = "t" in mi
    t = _vec(mi, "t", n) if has_t else []
    fill = _vec(mi, "l_fill", n - 1, default=0)
    for i in range(n - 1):
        if fill[i] < 0:
            raise Exception(f"Member {mi['name']}: ballast level in section {i+1} is negative.")
        if fill[i] > st[i + 1] - st[i]:
            raise Exception(f"Member {mi['name']}: ballast level in section {i+1} exceeds section length."
                            + f" ({fill[i]} > {st[i+1] - st[i]}).")
    rf = mi.get("rho_fill", 1025)
    if not isinstance(rf, (list, tuple, np.ndarray)):
        rho_fill = [float(rf)] * (n - 1)
    elif len(rf) == n - 1:
        rho_fill = [float(x) for x in rf]
    else:
        raise Exception(f"Member {mi['name']}: the number of provided ballast densities (rho_fill) must be 1 "
                        "less than the number of stations.")
    cs = mi.get("cap_stations", [])
    cap_st = [float(x) for x in np.atleast_1d(cs)]
    nc = len(cap_st)
    cap_t = _vec(mi, "cap_t", nc) if nc else []
    cap_d = _vec(mi, "cap_d_in", nc) if nc else []
    head = [int(mi["type"]), 1.0 if circ else 0.0, 1.0 if potMod else 0.0, 1.0 if mcf else 0.0,
            1.0 if str(mi["name"]) == "nacelle" else 0.0, n, nc, len(heads), 1.0 if has_t else 0.0,
            float(_scalar(mi, "gamma", 0.0)), dlsMax, float(_scalar(mi, "rho_shell", 8500.))]
    return (head + [float(x) for x in mi["rA"]] + [float(x) for x in mi["rB"]] + list(heads) + st + dd + t + fill
            + rho_fill + _vec(mi, "Cd_q", n, 0.0) + _vec(mi, "Cd", n, 0.6, 0) + _vec(mi, "Cd", n, 0.6, 1)
            + _vec(mi, "CdEnd", n, 0.6) + _vec(mi, "Ca_q", n, 0.0) + _vec(mi, "Ca", n, 0.97, 0)
            + _vec(mi, "Ca", n, 0.97, 1) + _vec(mi, "CaEnd", n, 0.6) + cap_st + cap_t + cap_d)


def design_spec(design, r6=None, statics=None, heading_adjust=0.0):
    """The spec record of one single-FOWT design (layout: csrc/rh_prep.h).  statics: the
    FOWT.setStatics entries that override the computed ones (and C_moor, MoorPy's stiffness)."""
    head, blocks, rots = _spec_parts(design, r6, statics, heading_adjust)
    return np.concatenate([head, np.asarray([x for blk in blocks for x in blk], dtype=float),
                           np.asarray(rots, dtype=float).ravel()])


def _spec_parts(design, r6, statics, heading_adjust):
    """design_spec in pieces: (header + given statics, one value list per member entry, rotor
    rows); the member blocks follow the header back to back, in platform-member order."""
    site, plat = design["site"], design["platform"]
    rho = get_from_dict(site, "rho_water", default=1025.0)
    g = get_from_dict(site, "g", default=9.81)
    potModMaster = get_from_dict(plat, "potModMaster", dtype=int, default=0)
    dlsMax = get_from_dict(plat, "dlsMax", default=5.0)
    blocks = []
    nmemb = 0
    for mi in plat["members"]:
        hd = mi.get("heading", 0.0)
        hd = hd if isinstance(hd, (list, tuple, np.ndarray)) else [hd]
        blocks.append(_member_spec(mi, [float(h) + heading_adjust for h in hd], dlsMax, potModMaster, True))
        nmemb += 1
    rots = []
    turb = design.get("turbine")
    if turb:
        nrot = get_from_dict(turb, "nrotors", dtype=int, shape=0, default=1)
        for key in ("tower", "nacelle"):
            ms = turb.get(key)
            if ms is not None:
                for mem in (ms if isinstance(ms, list) else [ms] * nrot):
                    blocks.append(_member_spec(mem, [0.0], 5.0, 0, False))
                    nmemb += 1
        hhub = np.atleast_1d(get_from_dict(turb, "hHub", shape=-1, default=100.0))
        if np.any(hhub < 0):
            raise NotImplementedError("underwater rotors are outside the accelerated path")
        if all(k in turb for k in ("mRNA", "IxRNA", "IrRNA", "xCG_RNA", "overhang", "shaft_tilt")):
            # the RNA inputs (raft/statics.py RNA.__init__, raft/raft_rotor.py:42-111); the hub
            # height correction r_rel[2] = hHub - q_z overhang is applied in rh_prep.h
            if "rRNA" in turb:
                rr = get_from_dict(turb, "rRNA", shape=[nrot, 3])
            elif nrot > 1:
                raise Exception("For designs with more than one rotor, the RNA reference point must be specified "
                                "for each of them.")
            else:
                rr = [[0.0, 0.0, 100.0]]
            cols = [_vec(turb, k, nrot) for k in ("mRNA", "IxRNA", "IrRNA", "xCG_RNA", "overhang")]
            tilt, toe = _vec(turb, "shaft_tilt", nrot), _vec(turb, "shaft_toe", nrot, 0)
            yaw = _vec(turb, "yaw_mode", nrot, 0)
            hh = _vec(turb, "hHub", nrot) if "hHub" in turb else [0.0] * nrot
            for ir in range(nrot):
                rots.append([c[ir] for c in cols] + [tilt[ir] * np.pi / 180, toe[ir] * np.pi / 180, int(yaw[ir]),
                                                     *[float(x) for x in rr[ir]], 1.0 if "hHub" in turb else 0.0,
                                                     hh[ir]])
        elif nrot:
            if not statics or not all(k in statics for k in ("M_struc", "C_struc", "C_hydro")):
                raise ValueError("turbine: mRNA, IxRNA, IrRNA, xCG_RNA, overhang and shaft_tilt are required")
    statics = dict(statics or {})
    moor = design.get("mooring")
    if moor and "C_moor" not in statics:
        # this FOWT's own mooring stiffness at the pose (raft/fowt.py setPosition with
        # raft/mooring.py, MoorPy in the reference: raft/raft_fowt.py:166-189, 275-288)
        from .mooring import MooringSystem
        ms = MooringSystem.from_yaml(moor)
        ms.transform(trans=[0.0, 0.0], rot=heading_adjust)
        ms.initialize()
        ms.set_body_positions([np.zeros(6) if r6 is None else np.asarray(r6, dtype=float)])
        statics["C_moor"] = ms.coupled_stiffness_analytic()
    hdr = [MAGIC, nmemb, len(rots), rho, g, *(np.zeros(6) if r6 is None else np.asarray(r6, dtype=float)),
           *[1.0 if k in statics else 0.0 for k in STATIC_KEYS]]
    given = [np.asarray(statics[k], dtype=float).ravel() for k in STATIC_KEYS if k in statics]
    return np.concatenate([np.asarray(hdr, dtype=float), *given]), blocks, rots


class SweepSpecs:
    """sweep_specs with the base design parsed once: records(mults) gives the spec records of
    those variants (the per-block call of a pipelined sweep, raft/batch.py solve_sweep)."""

    def __init__(self, base, r6=None, statics=None):
        self.base, self.r6, self.statics = base, r6, statics
        self._parts = _sweep_base(base, r6, statics)

    def records(self, mults):
        return sweep_specs(self.base, mults, self.r6, self.statics, _parts=self._parts)


def _sweep_base(base, r6, statics):
    """The base record of a sweep and the slots (offsets) of the fields the sweep edits."""
    head, blocks, rots = _spec_parts(base, r6, statics, 0.0)
    spec0 = np.concatenate([head, np.asarray([x for blk in blocks for x in blk], dtype=float),
                            np.asarray(rots, dtype=float).ravel()])
    plat = base["platform"]["members"]
    slots, off = [], len(head)
    for i, blk in enumerate(blocks):
        if i < 4:
            n, nh, circ = int(blk[5]), int(blk[7]), blk[1] != 0.0
            o_r = off + 12                          # head (12), then rA (3), rB (3), heads, stations
            o_d = o_r + 6 + nh + n
            slots.append((o_r, o_d, n, circ))
        off += len(blk)
    if len(slots) < 4 or len(plat) < 4:
        raise ValueError("sweep_specs: the sweep edits four platform members")
    return spec0, slots


def sweep_specs(base, mults, r6=None, statics=None, _parts=None):
    """The spec records of parametersweep variants of `base` (raft/sweep.py sweep_variant with
    each row of `mults`), without building a design dict per variant: the base record is
    flattened once, and per variant only the fields the sweep edits -- rA, rB and d of the
    first four platform members (raft/sweep.py variant_members) -- are rewritten in place,
    with the same parsing (_vec / _pairs) design_spec applies.  Equal, value for value, to
    design_spec(sweep_variant(base, m)) (tests/test_native_prep.py)."""
    from .sweep import variant_members
    spec0, slots = _parts if _parts is not None else _sweep_base(base, r6, statics)
    M = np.atleast_2d(np.asarray(mults, dtype=float))
    fast = _variant_fields(base, M, slots)
    if fast is not None:      # every variant at once: the assignments of variant_members on columns
        S = np.tile(spec0, (len(M), 1))
        for (o_r, o_d, n, circ), (rA, rB, dcols) in zip(slots, fast):
            S[:, o_r:o_r + 3] = rA
            S[:, o_r + 3:o_r + 6] = rB
            S[:, o_d:o_d + dcols.shape[1]] = dcols
        return list(S)
    out = []
    for m in M:
        s = spec0.copy()
        for (o_r, o_d, n, circ), mi in zip(slots, variant_members(base, m)):
            s[o_r:o_r + 3] = [float(x) for x in mi["rA"]]
            s[o_r + 3:o_r + 6] = [float(x) for x in mi["rB"]]
            dd = _vec(mi, "d", n) if circ else _pairs(mi, "d", n)
            s[o_d:o_d + len(dd)] = dd
        out.append(s)
    return out


def _variant_fields(base, M, slots):
    """raft/sweep.py variant_members for every row of M at once: per edited member (rA [nd, 3],
    rB [nd, 3], the parsed d entries [nd, ...]), the same floating-point operations in the same
    order, column-wise.  None when the base layout is not the one it restates (columns 0 and 1
    circular with scalar d, the pontoon rectangular with a [w, h] pair, member 3's d unchanged):
    sweep_specs then edits each variant's members one by one."""
    from .sweep import SWEEP_VARIABLES, sweep_baseline
    mem = base["platform"]["members"]
    circ = [c for _, _, _, c in slots]
    scalar_d = all(not isinstance(mem[i]["d"], (list, tuple, np.ndarray)) for i in (0, 1))
    pair = isinstance(mem[2]["d"], (list, tuple, np.ndarray)) and len(mem[2]["d"]) == 2 and \
        not isinstance(mem[2]["d"][0], (list, tuple, np.ndarray))
    if not (circ[0] and circ[1] and not circ[2] and scalar_d and pair):
        return None
    bl = sweep_baseline(base)
    a, b, c, dd, e = (bl[k] * M[:, i] for i, k in enumerate(SWEEP_VARIABLES))
    nd = len(M)
    rA = [np.tile(np.asarray([float(x) for x in mem[i]["rA"]]), (nd, 1)) for i in range(4)]
    rB = [np.tile(np.asarray([float(x) for x in mem[i]["rB"]]), (nd, 1)) for i in range(4)]
    pd1 = float(mem[2]["d"][1])
    rA[2][:, 0] = rA[2][:, 0] * (a / bl["ccD"])                 # centre-column diameter
    rA[3][:, 0] = rA[3][:, 0] * (a / bl["ccD"])
    rB[2][:, 0] = rA[1][:, 0] - b / 2                           # outer-column diameter
    rB[3][:, 0] = rB[1][:, 0] - b / 2
    rA[0][:, 2] = c                                             # draft
    rA[1][:, 2] = c
    rA[2][:, 2] = c + pd1 / 2
    rB[2][:, 2] = c + pd1 / 2
    rA[1][:, 0] = dd                                            # outer-column radius
    rB[1][:, 0] = dd
    rB[2][:, 0] = dd - b / 2
    rB[3][:, 0] = dd - b / 2
    rA[2][:, 2] = rA[0][:, 2] + e / 2                           # pontoon height
    rB[2][:, 2] = rA[1][:, 2] + e / 2
    n = [sl[2] for sl in slots]
    d0 = np.repeat(a[:, None], n[0], axis=1)
    d1 = np.repeat(b[:, None], n[1], axis=1)
    d2 = np.tile(np.stack([np.full(nd, float(mem[2]["d"][0])), e], axis=1), (1, n[2]))
    m3 = mem[3]
    d3 = np.tile(np.asarray(_vec(m3, "d", n[3]) if circ[3] else _pairs(m3, "d", n[3]), dtype=float), (nd, 1))
    return list(zip(rA, rB, [d0, d1, d2, d3]))


class PreparedDesigns:
    """Host tables of many designs from one rh_prep_designs call: `packed` (every design's
    real-valued tables back to back, the layout of raft/prep.py host_tables), `mstart`,
    and per design (offset, length, mstart offset, nn, nm) in `info`; `statics` [nd, 5, 6, 6]
    = M_struc, B_struc, C_struc, C_hydro, A_hydro_morison.
    pinned: write `packed` and `mstart` into one page-locked host tensor (`pinned`, packed
    then mstart as int32 bytes) so that they go up in one asynchronous copy
    (raft/batch.py DesignBatch._upload); torch's pinned-memory cache recycles it only after
    that copy has run."""

    def __init__(self, specs, w, k, nthreads=0, pinned=False):
        L = N.lib()
        nd = len(specs)
        off = np.zeros(nd + 1, dtype=np.int64)
        off[1:] = np.cumsum([len(s) for s in specs])
        flat = np.ascontiguousarray(np.concatenate(specs) if nd else np.zeros(0))
        w = np.ascontiguousarray(w, dtype=float)
        k = np.ascontiguousarray(k, dtype=float)
        h = ctypes.c_void_p()
        N.check(L.rh_prep_designs(nd, flat.ctypes.data, off.ctypes.data, len(w), w.ctypes.data, k.ctypes.data,
                                  int(nthreads), ctypes.byref(h)), "rh_prep_designs")
        try:
            info = np.zeros(5 * nd + 2, dtype=np.int64)
            N.check(L.rh_prep_layout(h, info.ctypes.data), "rh_prep_layout")
            npk, nms = int(info[5 * nd]), int(info[5 * nd + 1])
            self.pinned = None
            if pinned:
                import torch
                self.pinned = torch.empty(npk + (nms + 1) // 2, dtype=torch.float64, pin_memory=True)
                buf = self.pinned.numpy()
                self.packed = buf[:npk]
                self.mstart = buf[npk:].view(np.int32)[:nms]
            else:
                self.packed = np.empty(npk, dtype=float)
                self.mstart = np.empty(nms, dtype=np.int32)
            self.statics = np.empty([nd, 5, 6, 6], dtype=float)
            N.check(L.rh_prep_copy(h, self.packed.ctypes.data, self.mstart.ctypes.data, self.statics.ctypes.data),
                    "rh_prep_copy")
            # MacCamy-Fuchs designs: their [nn][9][nw] inertia tables (raft/prep.py node_table)
            self.imat = {}
            for i in range(nd):
                n = L.rh_prep_imat(h, i, None)
                N.check(0 if n >= 0 else int(n), "rh_prep_imat")
                if n > 0:
                    a = np.empty(int(n), dtype=complex)
                    L.rh_prep_imat(h, i, a.ctypes.data)
                    self.imat[i] = a.reshape(int(info[5 * i + 3]), 9, len(w))
        finally:
            L.rh_prep_free(h)
        self.info = info[:5 * nd].reshape(nd, 5)
        self.nd = nd
        self.nw = len(w)
        self._layouts = {}

    def __len__(self):
        return len(self.info)

    def host_tables(self, i):
        """Design i's tables in the form of raft/prep.py host_tables (views of `packed`)."""
        o, n, mo, nn, nm = (int(x) for x in self.info[i])
        cached = self._layouts.get((nn, nm))
        if cached is None:                          # one layout per (nodes, members) shape
            nw = self.nw
            shapes = [("w", (nw,)), ("k", (nw,)), ("node", (N.NF_COUNT, max(nn, 1))),
                      ("memb", (N.MF_COUNT, max(nm, 1))), ("M", (6, 6)), ("B", (6, 6)), ("C", (6, 6))]
            layout, off = {}, 0
            for name, shp in shapes:
                layout[name] = (off, shp)
                off += int(np.prod(shp))
            cached = self._layouts[(nn, nm)] = (layout, off)
        layout, total = cached
        assert total == n
        return dict(packed=self.packed[o:o + n], layout=layout, imat=self.imat.get(i), mstart=self.mstart[mo:mo + nm + 1],
                    nn=nn, nm=nm, per_bin=False)
