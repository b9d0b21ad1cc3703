"""ctypes binding of librafthip.so (include/rafthip.h).

This is the drop-in boundary: the reference has no FFI, so the binding
a maintainer adds on the reference side is exactly this module.
There is no CPU fallback: importing the product on a machine without the built library
or without a visible GPU raises at the first call that needs the device.
"""
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RAFTHIP_LIB", os.path.join(os.path.dirname(_HERE), "librafthip.so"))

RH_OK, RH_EINVAL, RH_ENAN, RH_ESINGULAR, RH_EHIP = 0, -1, -2, -3, -4
RH_QTF_INCIDENT_CACHED = 1
RH_CASE_CONVERGED, RH_CASE_NOT_CONVERGED, RH_CASE_NAN, RH_CASE_SINGULAR = 1, 0, -2, -3
SPECTRUM_CODES = {"JONSWAP": 0, "unit": 1, "constant": 2, "none": 3, "still": 3}

# node-table field order (enum rh_node_field)
NODE_FIELDS = ["RX", "RY", "RZ", "XX", "XY", "XZ", "QX", "QY", "QZ", "P1X", "P1Y", "P1Z", "P2X", "P2Y", "P2Z",
               "AQ", "AP1", "AP2", "AEND", "CDQ", "CDP1", "CDP2", "CDEND", "CIRC", "AI", "MCF",
               "I00", "I01", "I02", "I10", "I11", "I12", "I20", "I21", "I22", "T"]
NF = {name: i for i, name in enumerate(NODE_FIELDS)}
NF_COUNT = len(NODE_FIELDS)
MF_COUNT = 21   # enum rh_member_field: cq[6], c1[6], c2[6], |q|^2, |p1|^2, |p2|^2

_p = ctypes.c_void_p


class RhDesign(ctypes.Structure):
    _fields_ = [("nw", ctypes.c_int), ("nn", ctypes.c_int), ("nhead", ctypes.c_int), ("mb_per_bin", ctypes.c_int),
                ("dw", ctypes.c_double), ("depth", ctypes.c_double), ("rho", ctypes.c_double), ("g", ctypes.c_double),
                ("pdyn_rho_g", ctypes.c_double),
                ("w", _p), ("k", _p), ("node", _p), ("nm", ctypes.c_int), ("memb", _p), ("mstart", _p),
                ("imat_mcf", _p), ("uhat", _p), ("finer", _p), ("kproj", _p),
                ("M", _p), ("B", _p), ("C", _p)]


class RhCases(ctypes.Structure):
    _fields_ = [("ncase", ctypes.c_int), ("design", _p), ("head", _p), ("spectrum", _p),
                ("Hs", _p), ("Tp", _p), ("gamma", _p), ("nIter", ctypes.c_int),
                ("XiStart", ctypes.c_double), ("tol", ctypes.c_double), ("fext", _p), ("order", _p),
                ("Xi_init", _p), ("first_iter", ctypes.c_int), ("group_start", _p), ("ngroup", ctypes.c_int)]


class RhSolveOut(ctypes.Structure):
    _fields_ = [("Xi", _p), ("Xi_last", _p), ("iters", _p), ("status", _p), ("zeta", _p), ("B_drag", _p),
                ("Bmat", _p), ("psd", _p), ("std", _p), ("rao", _p), ("Z", _p), ("Xi_prev", _p), ("margin", _p),
                ("F_wave", _p)]


class RhQtfDesign(ctypes.Structure):
    _fields_ = [("n2", ctypes.c_int), ("nq", ctypes.c_int), ("nmq", ctypes.c_int), ("nkr", ctypes.c_int),
                ("beta", ctypes.c_double), ("depth", ctypes.c_double), ("rho", ctypes.c_double), ("g", ctypes.c_double),
                ("w2", _p), ("k2", _p), ("qnode", _p), ("qmemb", _p), ("qmstart", _p), ("kstart", _p),
                ("kray", _p), ("hank", _p), ("order", ctypes.c_int)]


class NativeError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()


def lib():
    """Load librafthip.so once; raise loudly if it is missing (no fallback path)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise NativeError(f"librafthip.so not found at {LIB_PATH}: build it with "
                                  "`python -c 'import __graft_entry__ as g; g.build()'`")
            # torch first: its bundled HIP runtime has the same SONAME (libamdhip64.so.7) as the
            # one librafthip links, so loading torch first makes both share ONE runtime.  Loaded
            # the other way round, torch brings a second HIP/HSA runtime into the process and
            # the library's hipGetDeviceCount finds no device.
            import torch  # noqa: F401
            L = ctypes.CDLL(LIB_PATH)
            L.rh_last_error.restype = ctypes.c_char_p
            for name, args in {
                "rh_ctx_create": [ctypes.c_int, ctypes.POINTER(_p)],
                "rh_ctx_destroy": [_p],
                "rh_wave_tables": [_p, ctypes.POINTER(RhDesign), _p, _p, _p, _p, _p],
                "rh_wave_tables_batch": [_p, ctypes.POINTER(RhDesign), ctypes.c_int, _p, ctypes.c_int, _p],
                "rh_solve_cases": [_p, ctypes.POINTER(RhDesign), ctypes.c_int, ctypes.POINTER(RhCases),
                                   ctypes.POINTER(RhSolveOut), _p],
                "rh_heading_response": [_p, ctypes.POINTER(RhDesign), ctypes.c_int, ctypes.c_int, _p, _p, _p, _p,
                                        _p, _p, _p],
                "rh_heading_response_ext": [_p, ctypes.POINTER(RhDesign), ctypes.c_int, ctypes.c_int, _p, _p, _p,
                                            _p, _p, ctypes.c_int, _p, _p, _p],
                "rh_linearize": [_p, ctypes.POINTER(RhDesign), ctypes.c_int, _p, _p, _p, _p, _p, _p],
                "rh_drag_excitation": [_p, ctypes.POINTER(RhDesign), ctypes.c_int, _p, _p, _p, _p],
                "rh_lin_partial_sums": [_p, ctypes.POINTER(RhDesign), ctypes.c_int, _p, _p, ctypes.c_int, ctypes.c_int,
                                        _p, _p],
                "rh_bin_step": [_p, ctypes.POINTER(RhDesign), ctypes.c_int, _p, _p, _p, ctypes.c_double, ctypes.c_int,
                                ctypes.c_int, _p, _p, _p, _p, _p, _p],
                "rh_sea_state": [_p, ctypes.c_int, ctypes.c_int, _p, ctypes.c_double, _p, _p, _p, _p, _p, _p, _p],
                "rh_motion_stats": [_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, _p, _p, _p, _p],
                "rh_system_solve": [_p, ctypes.c_int, ctypes.c_int, _p, _p, _p, _p, _p],
                "rh_system_solve_batch": [_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _p, _p, _p, _p, _p],
                "rh_array_response": [_p, ctypes.POINTER(RhDesign), ctypes.c_int, ctypes.c_int, ctypes.c_int, _p, _p,
                                      _p, _p, _p, _p, _p, _p],
                "rh_array_response_stats": [_p, ctypes.POINTER(RhDesign), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            _p, _p, _p, _p, _p, _p, _p, ctypes.c_double, _p, _p, _p, _p],
                "rh_array_solve_stats": [_p, ctypes.POINTER(RhDesign), ctypes.c_int, ctypes.c_int, ctypes.c_int, _p, _p,
                                         _p, _p, ctypes.c_double, _p, _p, _p],
                "rh_wave_excitation": [_p, ctypes.POINTER(RhDesign), ctypes.c_int, ctypes.c_int, _p, _p, _p, _p, _p,
                                       _p],
                "rh_channel_stats": [_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, _p,
                                     _p, ctypes.c_int, _p, _p, _p, _p],
                "rh_qtf_slender": [_p, ctypes.POINTER(RhQtfDesign), ctypes.c_int, _p, _p, _p, _p, _p,
                                   ctypes.c_longlong, _p],
                "rh_qtf_slender_ext": [_p, ctypes.POINTER(RhQtfDesign), ctypes.c_int, _p, _p, _p, _p, _p,
                                       ctypes.c_longlong, ctypes.c_int, _p],
                "rh_qtf_slender_rows": [_p, ctypes.POINTER(RhQtfDesign), ctypes.c_int, _p, _p, _p, ctypes.c_int,
                                        ctypes.c_int, _p, _p, ctypes.c_longlong, _p],
                "rh_qtf_hermitian_fill": [_p, ctypes.c_int, _p, _p],
                "rh_set_solver": [_p, ctypes.c_int],
                "rh_set_a0": [_p, ctypes.c_int],
                "rh_set_qtf_waves": [_p, ctypes.c_int],
                "rh_set_qtf_path": [_p, ctypes.c_int],
                "rh_qtf_hankel": [_p, ctypes.c_int, _p, ctypes.c_int, _p, _p, _p],
                "rh_force_2nd": [_p, ctypes.c_int, _p, _p, ctypes.c_int, _p, ctypes.c_double, _p, _p, _p, _p],
                "rh_force_2nd_batch": [_p, ctypes.c_int, ctypes.c_int, _p, _p, ctypes.c_int, _p, ctypes.c_int, _p,
                                       ctypes.c_double, _p, _p, _p, _p],
                "rh_force_2nd_spectrum": [_p, ctypes.c_int, _p, _p, ctypes.c_int, _p, ctypes.c_double, _p, _p, _p, _p,
                                          _p],
                "rh_prep_designs": [ctypes.c_int, _p, _p, ctypes.c_int, _p, _p, ctypes.c_int, ctypes.POINTER(_p)],
                "rh_prep_layout": [_p, _p],
                "rh_prep_copy": [_p, _p, _p, _p],
                "rh_qtf_tables": [ctypes.c_int, _p, ctypes.c_longlong, ctypes.c_double, _p, ctypes.c_longlong, _p,
                                  ctypes.c_longlong, _p],
            }.items():
                fn = getattr(L, name)
                fn.argtypes = args
                fn.restype = ctypes.c_int
            L.rh_prep_free.argtypes = [_p]
            L.rh_prep_free.restype = None
            L.rh_prep_imat.argtypes = [_p, ctypes.c_int, _p]
            L.rh_prep_imat.restype = ctypes.c_longlong
            L.rh_version.restype = ctypes.c_int
            L.rh_group_cases.argtypes = []
            L.rh_group_cases.restype = ctypes.c_int
            L.rh_solve_noxi_max_bins.argtypes = []
            L.rh_solve_noxi_max_bins.restype = ctypes.c_int
            L.rh_qtf_workspace_bytes.argtypes = [ctypes.POINTER(RhQtfDesign)]
            L.rh_qtf_workspace_bytes.restype = ctypes.c_longlong
            _lib = L
    return _lib


def check(rc, what=""):
    """Map a C-ABI return code onto the reference's exception types."""
    if rc == RH_OK:
        return
    msg = lib().rh_last_error().decode(errors="replace")
    if rc == RH_EINVAL:
        raise ValueError(f"{what}: {msg}")
    if rc == RH_ENAN:
        raise Exception("Nan detected in response vector Xi.")   # raft/raft_model.py:957
    if rc == RH_ESINGULAR:
        raise np.linalg.LinAlgError("Singular matrix")
    raise NativeError(f"{what}: {msg}")


_ctx = {}


def context(device=0):
    """Per-(thread, device) library context (the ABI is thread-compatible, not thread-safe)."""
    key = (threading.get_ident(), device)
    c = _ctx.get(key)
    if c is None:
        h = _p()
        check(lib().rh_ctx_create(device, ctypes.byref(h)), "rh_ctx_create")
        c = _ctx[key] = h
    return c


def ptr(t):
    """Device pointer of a torch tensor (or None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("device tensor expected")
    if not t.is_contiguous():
        raise ValueError("contiguous tensor expected")
    return ctypes.c_void_p(t.data_ptr())


def stream_handle(torch, device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
