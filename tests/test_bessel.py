"""CPU check of the device Bessel restatement (raft-teststuff_amd/csrc/rh_bessel.h, the Kim &
Yue Hankel table of raft/raft_member.py:1104-1107) against scipy.special.hankel1, the
function the reference calls: the header is compiled for the host with g++ (tools/
bessel_host.cpp) and evaluated over the arguments k R the QTF grids produce and beyond."""
import ctypes
import os
import subprocess
import tempfile

import numpy as np
import pytest
from scipy.special import hankel1

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    out = os.path.join(tempfile.mkdtemp(), "bessel_host.so")
    subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-o", out, os.path.join(ROOT, "tools", "bessel_host.cpp")],
                   check=True)
    L = ctypes.CDLL(out)
    L.rh_hankel_deriv_host.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    return L


def table(L, x):
    x = np.ascontiguousarray(x, dtype=float)
    out = np.zeros([len(x), 12, 2])
    L.rh_hankel_deriv_host(len(x), x.ctypes.data, out.ctypes.data)
    return out[..., 0] + 1j * out[..., 1]


def reference(x):
    H = hankel1(np.arange(-1, 13)[:, None], np.asarray(x)[None, :])
    return (0.5 * (H[0:12] - H[2:14])).T


@pytest.mark.parametrize("lo,hi", [(1e-3, 2.0), (2.0, 14.0), (14.0, 80.0), (80.0, 400.0)])
def test_hankel_derivative_table_matches_scipy(lib, lo, hi):
    x = np.geomspace(lo, hi, 3000)
    got, ref = table(lib, x), reference(x)
    err = np.abs(got - ref) / np.abs(ref)
    assert err.max() < 1e-13, (err.max(), x[np.unravel_index(err.argmax(), err.shape)[0]])


def test_branch_boundaries(lib):
    """Continuity at the series / recurrence switch (x = 2) and exact zeros of J0, J1."""
    x = np.array([2.0 - 1e-12, 2.0, 2.0 + 1e-12, 2.404825557695773, 3.831705970207512, 5.520078110286311])
    err = np.abs(table(lib, x) - reference(x)) / np.abs(reference(x))
    assert err.max() < 1e-13, err.max()
