"""Design x sea-state batches: the C5 throughput path (BASELINE.json configs[4]).

The reference evaluates a design sweep as one runRAFT per design and one solveDynamics per
case (raft/parametersweep.py:91, raft/raft_model.py:244-388).  Here every design is
prepared once on the host (members, statics, added mass: raft/member.py, raft/statics.py)
and on the device (node tables, per-heading wave tables), and then ALL (design, sea state)
cases go through one rh_solve_cases launch, one workgroup per case, sorted by
(design, heading) so an XCD streams one design's tables out of its L2.

Multi-GPU: designs are dealt to ranks in contiguous blocks (each rank prepares only its
own designs, so the host preparation scales with the rank count too); the per-case
outputs are all-gathered once at the end (raft/parallel.py gather_cases).
"""
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from .hydro_math import get_from_dict
from .model import Model
from .second_order import solve_batch_2nd
from .solver import CaseSet


class DesignBatch:
    """Prepared single-FOWT designs sharing one frequency grid.

    designs : list of design dicts (each with `settings`, `site`, `platform`, `turbine`)
    statics : None, one dict for all designs, or one dict per design, of FOWT.setStatics
              entries (typically just {"C_moor": K}: the mooring stiffness MoorPy would give)
    r6      : platform pose for the linearisation (default: the reference position)
    """

    def __init__(self, designs, statics=None, r6=None, device=0, pool=None, light=False, native=False, specs=None,
                 threads=None, prepared=None):
        """pool: optional multiprocessing pool (see host_pool) that prepares the designs on
        the host in parallel; results are identical to the serial path.
        light: keep only what the device side needs of each design (HostDesign: its tables,
        grid and site scalars) instead of the full Model; from a pool this ships ~40 KB per
        design instead of ~150 KB of Python objects (the parent's unpickling was the cost).
        native: prepare every design in librafthip on host threads (raft/native_prep.py,
        rh_prep_designs; implies light): the pool, if any, only flattens the design dicts.
        specs: the designs' spec records, already flattened (native_prep.sweep_specs; implies
        native); `designs` then only supplies the site and the frequency grid.
        threads: host threads of the native preparation (default: the pool's size, else
        min(16, this process's cores)).
        prepared: the native preparation of exactly these designs, already made
        (prepare_native, e.g. on another host thread while the previous block solves; implies
        native)."""
        t0 = time.perf_counter()
        if isinstance(statics, dict) or statics is None:
            statics = [statics] * len(designs)
        if len(statics) != len(designs):
            raise ValueError("statics: one dict for all designs or one per design")
        self._prepared = None
        if native or specs is not None or light or prepared is not None:
            for d in {id(d): d for d in designs}.values():     # (a sweep passes one base dict many times)
                if get_from_dict((d or {}).get("platform") or {}, "potSecOrder", dtype=int, default=0) > 0:
                    raise NotImplementedError("DesignBatch: second-order loads (potSecOrder > 0) need the full design "
                                              "models (native=False, light=False): the QTFs are built there")
        if native or specs is not None or prepared is not None:
            P = prepared if prepared is not None else prepare_native(designs, statics, r6, pool, specs, threads)
            self.models = self._native(designs, P, device)
        else:
            jobs = [(d, st, r6, device, light) for d, st in zip(designs, statics)]
            if pool is not None and len(jobs) > 1:
                self.models = pool.map(prepare_design, jobs, chunksize=max(1, len(jobs) // (4 * pool._processes)))
            else:
                self.models = [prepare_design(j) for j in jobs]
        self.fowts = [m if isinstance(m, HostDesign) else m.fowtList[0] for m in self.models]
        m0 = self.models[0]
        for m in self.models[1:]:
            if m.nw != m0.nw or not np.array_equal(m.w, m0.w):
                raise ValueError("all designs of a batch must share the frequency grid")
            if m.nIter != m0.nIter or m.XiStart != m0.XiStart:
                raise ValueError("all designs of a batch must share nIter and XiStart")
        self.nIter, self.XiStart, self.nw, self.w = m0.nIter, m0.XiStart, m0.nw, m0.w
        self.host_seconds = time.perf_counter() - t0
        t0 = time.perf_counter()
        self.dds = self._upload(device)
        self.upload_seconds = time.perf_counter() - t0

    def _native(self, designs, P, device):
        """HostDesign-like records of natively prepared designs (prepare_native), holding
        views of the one packed host array."""
        if P.nd != len(designs):
            raise ValueError("DesignBatch: the native preparation is not one of these designs")
        self._prepared = P
        w, k, depth = P.w, P.k, P.depth
        st0 = designs[0].get("settings", {})
        nIter = get_from_dict(st0, "nIter", default=15, dtype=int)
        XiStart = get_from_dict(st0, "XiStart", default=0.1, dtype=float)
        sites = {}
        out = []
        for i, d in enumerate(designs):
            site = sites.get(id(d["site"]))
            if site is None:            # the site scalars once per distinct site (a sweep shares one)
                site = sites[id(d["site"])] = (get_from_dict(d["site"], "rho_water", default=1025.0),
                                               get_from_dict(d["site"], "g", default=9.81))
            out.append(NativeDesign(P, i, d, w, k, depth, nIter, XiStart, device, site=site))
        return out

    def _upload(self, device):
        """Every design's device tables in one host->device copy (plus one for the member
        ranges); each DeviceDesign holds views of its slices."""
        import torch
        from .prep import DeviceDesign, _torch
        _torch()
        dev = torch.device("cuda", device)
        if self._prepared is not None:     # native: already one packed host array
            P = self._prepared
            if getattr(P, "pinned", None) is not None:    # one asynchronous copy out of page-locked memory
                flat = P.pinned.to(dev, non_blocking=True)
                npk = P.packed.size
                packed = flat[:npk]
                mst = flat[npk:].view(torch.int32)[:P.mstart.size]
            else:
                packed = torch.from_numpy(P.packed).to(dev)
                mst = torch.from_numpy(P.mstart).to(dev)
            dds = []
            for i, f in enumerate(self.fowts):
                o, n, mo, nn, nm = (int(x) for x in P.info[i])
                f._dd = DeviceDesign(f, device=device, packed=packed[o:o + n], mstart=mst[mo:mo + nm + 1])
                dds.append(f._dd)
            return dds
        hs = [f.host_tables() for f in self.fowts]
        packed = torch.tensor(np.concatenate([h["packed"] for h in hs]), dtype=torch.float64, device=dev)
        mst = torch.tensor(np.concatenate([h["mstart"] for h in hs]).astype(np.int32), dtype=torch.int32, device=dev)
        dds, off, moff = [], 0, 0
        for f, h in zip(self.fowts, hs):
            n, k = h["packed"].size, h["mstart"].size
            f._dd = DeviceDesign(f, device=device, packed=packed[off:off + n], mstart=mst[moff:moff + k])
            dds.append(f._dd)
            off, moff = off + n, moff + k
        return dds

    def __len__(self):
        return len(self.models)

    def case_set(self, design_idx, cases):
        """CaseSet of (design index, case dict) pairs; one sea state per case."""
        return case_set_of(design_idx, cases)

    def case_set_grid(self, design_idx, state_idx, sea_states):
        """CaseSet of cases given as (design index, index into `sea_states`): a sweep's
        design x sea-state product without one case dict per case."""
        return case_set_grid(design_idx, state_idx, case_set_of(np.zeros(len(sea_states), dtype=np.int32), sea_states))

    def solve(self, design_idx, cases, tol=0.01, want=("psd", "std", "zeta", "B_drag"), prepared=None, out=None):
        """Drag fixed point + response of every case in one device call.  Returns the
        BatchResult (device tensors, stream-ordered): Xi [n,6,nw], iters, status, ...
        Case dicts with wind on an operating rotor (wind_speed > 0, turbine_status
        'operating', aeroServoMod > 0) get their design's aero-servo added mass and damping per
        bin, as runRAFT gives each case of a parametersweep design (raft/parametersweep.py:91,
        raft/raft_model.py:887-889): one CaseMB view per (design, distinct wind state) on the
        design's shared node and wave tables.  Such cases need the full design models
        (native=False, light=False): the rotors are built there.  out: preallocated outputs of
        a CaseSet batch (solver.solve_batch)."""
        if isinstance(cases, CaseSet):
            return solve_batch_2nd(self.dds, self.fowts, cases, self.nIter, self.XiStart, tol, want=want,
                                   prepared=prepared, out=out)
        cs = self.case_set(design_idx, cases)
        aero = self._aero_views(np.asarray(design_idx, dtype=np.int64), cases)
        if aero is None:
            return solve_batch_2nd(self.dds, self.fowts, cs, self.nIter, self.XiStart, tol, want=want,
                                   prepared=prepared)
        views, idx, owners = aero
        cs = CaseSet(idx, cs.heading, cs.spectrum, cs.Hs, cs.Tp, cs.gamma)
        return solve_batch_2nd(views, owners, cs, self.nIter, self.XiStart, tol, want=want)

    _WAVE_KEYS = ("wave_spectrum", "wave_period", "wave_height", "wave_heading", "wave_gamma", "iCase")

    def _aero_views(self, design_idx, cases):
        """(views, per-case view index, the FOWT of each view) when some case has an operating
        rotor, else None."""
        import torch
        from .model import CaseMB
        from .prep import linear_matrices
        hot = [i for i, c in enumerate(cases) if not isinstance(self.fowts[int(design_idx[i])], HostDesign)
               and Model._operating_rotor(self.fowts[int(design_idx[i])], c)]
        if not hot:
            for i, c in enumerate(cases):
                if get_from_dict(c, "wind_speed", shape=0, default=0.0) > 0 and \
                        isinstance(self.fowts[int(design_idx[i])], HostDesign):
                    raise NotImplementedError("DesignBatch: cases with wind need the full design models "
                                              "(native=False, light=False) to build the rotors")
            return None
        views = list(self.dds)
        owners = list(self.fowts)
        idx = design_idx.astype(np.int32).copy()
        made = {}
        heads = np.unique([float(np.atleast_1d(c.get("wave_heading", 0))[0]) for c in cases]) * np.pi / 180.0
        for i in hot:
            d = int(design_idx[i])
            c = cases[i]
            key = (d, tuple(sorted((k, str(v)) for k, v in c.items() if k not in self._WAVE_KEYS)))
            if key not in made:
                fowt = self.fowts[d]
                fowt.calcTurbineConstants(dict(c), ptfm_pitch=0)
                M, B, _, _ = linear_matrices(fowt)
                fowt.calcTurbineConstants(dict(c, wind_speed=0.0), ptfm_pitch=0)     # back to the aero-free design
                f64 = dict(dtype=torch.float64, device=self.dds[d].device)
                self.dds[d].ensure_headings(heads)
                views.append(CaseMB(self.dds[d], torch.tensor(M, **f64).contiguous(), torch.tensor(B, **f64).contiguous()))
                owners.append(fowt)
                made[key] = len(views) - 1
            idx[i] = made[key]
        return views, idx, owners


def case_set_of(design_idx, cases):
    """CaseSet of (design index, case dict) pairs; one sea state per case."""
    hd, sp, Hs, Tp, gm = [], [], [], [], []

    def one(c, k, dflt=None):
        v = c.get(k, dflt)
        if isinstance(v, (list, tuple, np.ndarray)):
            if len(v) != 1:
                raise NotImplementedError("DesignBatch: one sea state per case")
            return v[0]
        return v
    for c in cases:
        hd.append(float(one(c, "wave_heading", 0)))
        sp.append(str(one(c, "wave_spectrum", "JONSWAP")))
        Hs.append(float(one(c, "wave_height")))
        Tp.append(float(one(c, "wave_period")))
        gm.append(float(one(c, "wave_gamma", 0)))
    return CaseSet(np.asarray(design_idx, dtype=np.int32), hd, sp, Hs, Tp, gm)


def case_set_grid(design_idx, state_idx, cs0):
    """The CaseSet of cases (design index, index into the parsed sea states cs0)."""
    si = np.asarray(state_idx, dtype=np.int64)
    return CaseSet(np.asarray(design_idx, dtype=np.int32), cs0.heading[si], cs0.spectrum[si], cs0.Hs[si],
                   cs0.Tp[si], cs0.gamma[si])


def solve_sweep(designs, statics, design_idx, state_idx, sea_states, device=0, pool=None, chunks=4, tol=0.01,
                want=("psd", "std"), timings=None, specs=None, threads=None, first=1.0,
                last=1.0, block_path=True):
    """A design sweep solved in `chunks` design blocks, pipelined: while the device solves
    block k, the host prepares block k+1 (native preparation, raft/native_prep.py), so the
    host work hides behind the solve instead of preceding it.

    design_idx / state_idx: per case, its design (index into `designs`, non-decreasing: the
    design-major order of sweep_cases) and its sea state (index into `sea_states`).  Every
    case is solved exactly as in one DesignBatch call (per-case arithmetic, so the results are
    the same bits).  The uploads of a block go through a copy stream, so the host never
    waits behind a running solve; its sweep tables and its solve run on the current stream
    after an event on the uploads.  Returns (result dict of device tensors in case
    order, stream-ordered on the current stream; the per-block DesignBatches, kept alive
    with their tensors until the caller synchronises).  specs: optional spec records of the
    designs (native_prep.sweep_specs), or a function (a, b) -> the records of designs [a, b),
    called per block inside the pipeline (so their cost overlaps the previous block's solve).
    first, last: the first and last blocks' sizes relative to the others (the device idles
    while the first is prepared, and only the last block's solve runs after the host is done,
    so small ones shorten the pipeline's fill and drain; 1 = equal blocks, the default: on the
    C5 bench 0.25 / 0.5 measured within noise of it, 26.0-27.3 vs 25.5-27.5 ms).
    block_path: write each block's descriptors in one array (raft/sweep_block.py) instead of a
    DesignBatch of per-design objects (the same launches and bits; False: the per-design path).
    timings: optional list that receives,
    per block, the host seconds of (design preparation, case set + tables + uploads, solve
    enqueue, DesignBatch host part, DesignBatch upload part)."""
    import gc
    was = gc.isenabled()
    gc.disable()     # a full collection inside the pipeline stalled the host for 50-65 ms (profiles/r06_v1)
    try:
        return _solve_sweep(designs, statics, design_idx, state_idx, sea_states, device, pool, chunks, tol, want,
                            timings, specs, threads, first, last, block_path)
    finally:
        if was:
            gc.enable()


def _solve_sweep(designs, statics, design_idx, state_idx, sea_states, device, pool, chunks, tol, want, timings,
                 specs, threads, first, last, block_path=True):
    import torch
    from .solver import prepare_batch
    from .sweep_block import prepare_block
    design_idx = np.asarray(design_idx, dtype=np.int64)
    state_idx = np.asarray(state_idx, dtype=np.int64)
    if any(get_from_dict(c, "wind_speed", shape=0, default=0.0) > 0 for c in sea_states):
        raise NotImplementedError("solve_sweep: sea states with wind need the rotors of the full design models; "
                                  "use DesignBatch(designs, native=False).solve(design_idx, cases)")
    if np.any(np.diff(design_idx) < 0):
        raise ValueError("solve_sweep: cases must be design-major (non-decreasing design index)")
    nd = len(designs)
    cuts = sweep_cuts(nd, chunks, first, last)
    blocks = [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]
    dev = torch.device("cuda", device)
    compute = torch.cuda.current_stream(dev)
    copy = _copy_stream(dev)
    cs_all = case_set_of(np.zeros(len(sea_states), dtype=np.int32), sea_states)   # each sea state parsed once

    def prep(a, b):
        sp = None if specs is None else (specs(a, b) if callable(specs) else specs[a:b])
        st = statics if isinstance(statics, dict) or statics is None else statics[a:b]
        return prepare_native(designs[a:b], st, None, pool, sp, threads, pinned=True)

    # the sweep's outputs, allocated once: each block's solve writes its rows (no concatenation)
    nw = len(Model.frequency_grid(designs[0]))
    n = len(design_idx)
    c128 = dict(dtype=torch.complex128, device=dev)
    f64 = dict(dtype=torch.float64, device=dev)
    shapes = {"Xi": ([n, 6, nw], c128), "iters": ([n], dict(dtype=torch.int32, device=dev)),
              "status": ([n], dict(dtype=torch.int32, device=dev)), "zeta": ([n, nw], f64), "B_drag": ([n, 6, 6], f64),
              "psd": ([n, 6, nw], f64), "std": ([n, 6], f64), "rao": ([n, 6, nw], c128), "margin": ([n], f64)}
    full = {k: torch.empty(sh, **kw) for k, (sh, kw) in shapes.items()
            if k in ("iters", "status") or k in want or (k == "Xi" and "noXi" not in want)}
    parts, keep = [], []
    # The native preparation of block k+1 runs on a worker thread (rh_prep_designs releases the
    # GIL) while this thread uploads block k, tabulates it and enqueues its solve.
    with ThreadPoolExecutor(1) as ex:
        nxt = ex.submit(prep, *blocks[0]) if blocks else None
        for j, (a, b) in enumerate(blocks):
            lo, hi = np.searchsorted(design_idx, [a, b])
            t0 = time.perf_counter()
            P = nxt.result()
            tw = time.perf_counter() - t0
            nxt = ex.submit(prep, *blocks[j + 1]) if j + 1 < len(blocks) else None
            with torch.cuda.stream(copy):
                cs = case_set_grid(design_idx[lo:hi] - a, state_idx[lo:hi], cs_all)
                # the block's wave tables on the solve stream: beside the previous block's solve (on the
                # upload stream) they stretched each solve by 0.5 ms (profiles/r06_v3/c5_timeline.txt)
                fast = prepare_block(P, designs[a:b], cs, device, compute) if block_path else None
                if fast is not None:     # one descriptor array for the block (sweep_block.py)
                    B, prep_b = fast
                    t1 = time.perf_counter()
                else:
                    B = DesignBatch(designs[a:b], statics=statics if isinstance(statics, dict) or statics is None
                                    else statics[a:b], device=device, prepared=P)
                    t1 = time.perf_counter()
                    prep_b = prepare_batch(B.dds, cs, tables_stream=compute)
                ready = torch.cuda.Event()
                ready.record(copy)
            compute.wait_event(ready)
            t2 = time.perf_counter()
            res = B.solve(None, cs, tol=tol, want=want, prepared=prep_b,   # on the solve stream
                          out={k: v[lo:hi] for k, v in full.items()})
            if timings is not None:
                timings.append((t1 - t0, t2 - t1, time.perf_counter() - t2, getattr(B, "host_seconds", 0.0),
                                getattr(B, "upload_seconds", 0.0), tw))
            parts.append(res)
            keep.append((B, cs, prep_b, res))
    out = {k: full[k] if k in full else torch.cat([r[k] for r in parts], 0) for k in parts[0]}
    # The blocks' tables were allocated on the upload stream and are read by kernels on the
    # solve stream.  The caching allocator hands a freed block back to work on the stream that
    # allocated it, so order every later upload-stream operation after this sweep's kernels:
    # dropping `keep` before synchronising can then never let an upload overwrite tables that
    # a kernel is still reading.
    done = torch.cuda.Event()
    done.record(compute)
    copy.wait_event(done)
    return out, keep


def sweep_cuts(nd, chunks, first=1.0, last=1.0):
    """Block boundaries of a pipelined sweep over nd designs: `chunks` blocks, the first and
    the last weighted `first` and `last` against 1 for the others."""
    k = max(1, min(int(chunks), nd))
    wts = np.ones(k)
    if k > 1:
        wts[0], wts[-1] = first, last
    cuts = np.round(np.concatenate([[0.0], np.cumsum(wts)]) / wts.sum() * nd).astype(int)
    cuts[-1] = nd
    return np.maximum.accumulate(cuts)


_COPY_STREAMS = {}


def _copy_stream(dev):
    """One upload stream per device, kept across sweeps: the caching allocator keeps its
    blocks per stream, so a fresh stream per call would allocate every upload buffer anew."""
    import torch
    key = dev.index
    if key not in _COPY_STREAMS:
        _COPY_STREAMS[key] = torch.cuda.Stream(dev)
    return _COPY_STREAMS[key]


def prepare_native(designs, statics=None, r6=None, pool=None, specs=None, threads=None, pinned=False):
    """rh_prep_designs over every design (raft/native_prep.py): the host part of
    DesignBatch(native=True), callable on its own (a worker thread: the native call releases
    the GIL).  Returns the PreparedDesigns with the shared grid (w, k, depth) attached.
    pinned: its tables in page-locked memory (PreparedDesigns), uploaded asynchronously."""
    import os
    from .hydro_math import wave_numbers
    from .native_prep import PreparedDesigns
    t0 = time.perf_counter()
    if isinstance(statics, dict) or statics is None:
        statics = [statics] * len(designs)
    w = Model.frequency_grid(designs[0])
    depth = get_from_dict(designs[0]["site"], "water_depth", dtype=float)
    for d in designs[1:]:
        if d is designs[0]:
            continue
        if get_from_dict(d["site"], "water_depth", dtype=float) != depth or \
                not np.array_equal(Model.frequency_grid(d), w):
            raise ValueError("all designs of a batch must share the frequency grid and the site")
    k = wave_numbers(w, depth)
    if specs is None:
        jobs = [(d, None if r6 is None else np.asarray(r6, dtype=float), st) for d, st in zip(designs, statics)]
        if pool is not None and len(jobs) > 1:
            specs = pool.map(_spec_job, jobs, chunksize=max(1, len(jobs) // (4 * pool._processes)))
        else:
            specs = [_spec_job(j) for j in jobs]
    elif len(specs) != len(designs):
        raise ValueError("DesignBatch: one spec record per design")
    nt = threads or (pool._processes if pool is not None else min(16, len(os.sched_getaffinity(0))))
    P = PreparedDesigns(specs, w, k, nthreads=nt, pinned=pinned)
    P.w, P.k, P.depth = w, k, depth
    P.host_seconds = time.perf_counter() - t0
    return P


def prepare_design(job):
    """Host preparation of one single-FOWT design (members, statics, added mass and
    excitation coefficients at pose r6): the per-design part of runRAFT before the case loop
    (raft/raft_model.py:30-170, raft/raft_fowt.py:291-565, 848-880).  Pure NumPy, so it can
    run in a worker process; the device tables are built later by the caller."""
    d, st, r6, device = job[:4]
    light = len(job) > 4 and job[4]
    m = Model(d, statics=None if st is None else [st], device=device)
    if m.nFOWT != 1:
        raise NotImplementedError("DesignBatch handles single-FOWT designs (use Model for arrays)")
    f = m.fowtList[0]
    f.setPosition(np.zeros(6) if r6 is None else np.asarray(r6, dtype=float))
    f.calcStatics()
    f.calcHydroConstants()
    f.host_tables()            # the device-table layout, built here too (travels with the FOWT)
    return HostDesign(m) if light else m


class HostDesign:
    """What the device side needs of one prepared single-FOWT design: its host tables
    (prep.host_tables), frequency grid, site scalars and solver settings.  Stands in for the
    FOWT wherever only device_design() is used (DesignBatch light=True)."""

    def __init__(self, model):
        f = model.fowtList[0]
        self.nw, self.w, self.k, self.dw = f.nw, np.asarray(model.w), f.k, f.dw
        self.depth, self.rho_water, self.g = f.depth, f.rho_water, f.g
        self.nIter, self.XiStart = model.nIter, model.XiStart
        self.device_index = f.device_index
        self._host = f.host_tables()
        self._dd = None

    def host_tables(self):
        return self._host

    def device_design(self):
        if self._dd is None:
            from .prep import DeviceDesign
            self._dd = DeviceDesign(self, device=self.device_index)
        return self._dd

    def __getstate__(self):
        st = dict(self.__dict__)
        st["_dd"] = None
        return st


def _spec_job(job):
    from .native_prep import design_spec
    d, r6, st = job
    return design_spec(d, r6=r6, statics=st)


class NativeDesign(HostDesign):
    """HostDesign of a natively prepared design (rh_prep_designs): its tables are views of
    the batch's packed host array."""

    def __init__(self, P, i, design, w, k, depth, nIter, XiStart, device, site=None):
        self.nw, self.w, self.k, self.dw = len(w), w, k, w[1] - w[0]
        self.depth = depth
        if site is None:
            site = (get_from_dict(design["site"], "rho_water", default=1025.0),
                    get_from_dict(design["site"], "g", default=9.81))
        self.rho_water, self.g = site
        self.nIter, self.XiStart = nIter, XiStart
        self.device_index = device
        self._host = P.host_tables(i)
        self._dd = None


def _warm_worker(grids):
    from . import native_prep  # noqa: F401  (the spec writer of DesignBatch(native=True))
    from .hydro_math import wave_numbers
    for w, depth in grids:
        wave_numbers(w, depth)


def host_pool(processes, grids=()):
    """A pool of `processes` host workers for DesignBatch.  Create it BEFORE this process
    initialises the GPU (workers are started with 'spawn' and never touch the device).
    grids: (w, depth) pairs whose dispersion solutions each worker memoises up front (the
    per-site cost a sweep pays once, hydro_math.wave_numbers)."""
    import multiprocessing as mp
    return mp.get_context("spawn").Pool(processes, initializer=_warm_worker, initargs=(list(grids),))


def sweep_shard(design_idx, rank, world):
    """This rank's contiguous block [lo, hi) of a design-major case list and the design
    range [dlo, dhi) it touches (a design cut by a block boundary is prepared by both ranks)."""
    from .parallel import case_shard
    lo, hi = case_shard(len(design_idx), rank, world)
    if hi <= lo:
        return lo, hi, 0, 0
    return lo, hi, int(design_idx[lo]), int(design_idx[hi - 1]) + 1


def sweep_cases(n_designs, sea_states):
    """Every design paired with every sea state: (design index, case) lists, design-major."""
    idx = np.repeat(np.arange(n_designs, dtype=np.int32), len(sea_states))
    return idx, [dict(s) for _ in range(n_designs) for s in sea_states]
