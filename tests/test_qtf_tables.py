"""rh_qtf_tables (host C++, csrc/rh_qtf_host.h) against raft/qtf.py build_tables, the NumPy
statement of the same static QTF tables (raft/raft_fowt.py:1461-1625, raft/raft_member.py:
1111-1200): bit for bit, for designs with circular and rectangular members, Kim & Yue members,
displaced poses and several headings.  Host code only: runs without a GPU."""
import json
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DESIGNS = os.path.join(ROOT, "tests", "golden", "designs")


def _fowt(name, r6):
    import raft
    with open(os.path.join(DESIGNS, name + ".json")) as fh:
        design = json.load(fh)
    design["platform"]["outFolderQTF"] = None
    f = raft.Model(design, device=0).fowtList[0]
    f.setPosition(np.asarray(r6, dtype=float))
    return f


@pytest.fixture(scope="module")
def lib():
    import __graft_entry__ as g
    g.build()


@pytest.mark.parametrize("name", ["OC4semi-RAFT_QTF", "VolturnUS-S_example", "OC3spar"])
@pytest.mark.parametrize("r6", [np.zeros(6), [1.5, -0.7, 0.3, 0.01, -0.02, 0.05]])
def test_native_tables_equal_numpy_tables(lib, name, r6):
    from raft.hydro_math import wave_numbers
    from raft.qtf import build_tables, native_tables
    f = _fowt(name, r6)
    w2 = np.arange(0.04, 0.35, 0.01) * 2 * np.pi
    k2 = wave_numbers(w2, f.depth)
    for beta in (0.0, np.deg2rad(30.0), 1.234, -2.5):
        a = build_tables(f, w2, k2, beta)
        _, end, b = native_tables(f, beta)
        for k in ("qnode", "qmemb", "kray", "qmstart", "kstart"):
            np.testing.assert_array_equal(np.asarray(b[k]), np.asarray(a[k]), err_msg=f"{name} beta={beta} {k}")
        for k in ("rho", "g", "h"):
            assert b[k] == a[k]
    if name == "OC4semi-RAFT_QTF":
        assert b["kray"].shape[1] > 0      # Kim & Yue members exercised


def test_native_tables_into_a_buffer_at_an_offset(lib):
    from raft.qtf import native_tables, table_capacity
    f = _fowt("OC4semi-RAFT_QTF", np.zeros(6))
    _, n, ref = native_tables(f, 0.3)
    cap = table_capacity(f)
    assert n <= cap
    buf = np.full(37 + cap + 100, -7.0)
    _, end, t = native_tables(f, 0.3, buf, 37)
    assert end == 37 + n and np.all(buf[:37] == -7.0) and np.all(buf[end:] == -7.0)
    for k in ("qnode", "qmemb", "kray", "qmstart", "kstart"):
        np.testing.assert_array_equal(t[k], ref[k])
    with pytest.raises(ValueError):
        native_tables(f, 0.3, np.empty(cap - 1), 0)


def test_malformed_records_are_refused(lib):
    from raft import _native as N
    from raft.qtf import member_record
    f = _fowt("OC3spar", np.zeros(6))
    rec = np.concatenate([member_record(m) for m in f.memberList])
    out, iout, cnt = np.empty(100000), np.empty(100, dtype=np.int32), np.zeros(3, dtype=np.int32)
    L = N.lib()
    nm = len(f.memberList)

    def call(r, nmem=nm, cap=out.size, capi=iout.size):
        return L.rh_qtf_tables(nmem, r.ctypes.data, r.size, 0.0, out.ctypes.data, cap, iout.ctypes.data, capi,
                               cnt.ctypes.data)
    assert call(rec) == N.RH_OK
    assert call(rec[:-1]) == N.RH_EINVAL                       # truncated
    assert call(np.append(rec, 0.0)) == N.RH_EINVAL            # trailing data
    assert call(rec, nmem=nm + 1) == N.RH_EINVAL               # more members than records
    assert call(rec, cap=10) == N.RH_EINVAL                    # output too small
    assert call(rec, capi=1) == N.RH_EINVAL
    bad = rec.copy()
    bad[2] = 2.5                                               # non-integral node count
    assert call(bad) == N.RH_EINVAL
    assert "rh_qtf_tables" in L.rh_last_error().decode()
