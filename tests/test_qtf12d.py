"""potSecOrder=2 host side: the WAMIT .12d reader (raft/qtf_io.py read_qtf12d, FOWT.readQTF)
against the reference's own readQTF output on its example file
(examples/OC4semi-WAMIT_Coefs/marin_semi.12d; fixture tests/golden/qtf12d.npz, written by
tests/golden/make_golden.py qtf12d).  Bitwise: parsing, scaling and the Hermitian fill are
exact operations."""
import os

import numpy as np
import pytest

from conftest import load_golden
from raft.qtf_io import read_qtf12d, write_qtf12d


@pytest.fixture(scope="module")
def T():
    return load_golden("qtf12d")


def write_table(table, path):
    """An equivalent .12d text file of a numeric table (17 significant digits: loadtxt gives
    back the identical doubles)."""
    np.savetxt(path, table, fmt="%.17g")
    return path


def test_reader_matches_reference(T, tmp_path):
    for src in (T["table12d"], write_table(T["table12d"], str(tmp_path / "q.12d"))):
        h, w1, w2, q = read_qtf12d(src, float(T["rho"]), float(T["g"]))
        np.testing.assert_array_equal(h, T["heads_2nd"])
        np.testing.assert_array_equal(w1, T["w1_2nd"])
        np.testing.assert_array_equal(w2, T["w1_2nd"])
        np.testing.assert_array_equal(q, T["qtf"])


def test_reader_later_rows_win_and_mirror():
    """Row order semantics of the reference loop: a later row overrides an earlier one,
    including a row given for the mirrored (w2, w1) position."""
    rho, g = 1000.0, 10.0
    T1, T2 = 2 * np.pi / 0.5, 2 * np.pi / 1.0
    rows = np.array([[T1, T2, 0, 0, 1, 0, 0, 1.0, 2.0],
                     [T2, T1, 0, 0, 1, 0, 0, 3.0, 4.0],      # mirrored position, later: wins
                     [T1, T1, 0, 0, 4, 0, 0, 5.0, 0.0],
                     [T2, T2, 0, 0, 1, 0, 0, 6.0, 0.0]])
    h, w1, w2, q = read_qtf12d(rows, rho, g, ULEN=2)
    np.testing.assert_array_equal(w1, [0.5, 1.0])
    f = rho * g * 2
    assert q[1, 0, 0, 0] == f * (3 + 4j) and q[0, 1, 0, 0] == f * (3 - 4j)
    assert q[0, 0, 0, 3] == f * 2 * 5.0          # moments carry one more ULEN
    assert q[1, 1, 0, 0] == f * 6.0


def test_reader_rejects_bidirectional_and_ragged():
    r = np.array([[10.0, 10.0, 0, 30, 1, 0, 0, 1, 0]])
    with pytest.raises(ValueError, match="unidirectional"):
        read_qtf12d(r, 1025, 9.81)
    r = np.array([[10.0, 10.0, 0, 0, 1, 0, 0, 1, 0], [10.0, 20.0, 0, 0, 1, 0, 0, 1, 0]])
    with pytest.raises(ValueError, match="same values"):
        read_qtf12d(r, 1025, 9.81)


def test_reader_heading_lookup_mirrors_reference():
    """The reference matches the .12d heading column (degrees) against heads_2nd (radians,
    raft/raft_fowt.py:1676, 1686): heading 0 reads, any other heading raises IndexError from
    indhead[0].  Restated here on the reference's own loop semantics."""
    T1, T2 = 2 * np.pi / 0.5, 2 * np.pi / 1.0
    def rows(hd):
        return [[T1, T2, hd, hd, 1, 0, 0, 1.0, 2.0], [T2, T1, hd, hd, 1, 0, 0, 1.0, -2.0]]
    h, _, _, q = read_qtf12d(np.array(rows(0.0)), 1000.0, 10.0)
    assert h.tolist() == [0.0] and q[0, 1, 0, 0] == 1e4 * (1 + 2j)
    for heads in ([30.0], [0.0, 30.0]):
        rows_h = np.array([r for hd in heads for r in rows(hd)])
        with pytest.raises(IndexError):
            read_qtf12d(rows_h, 1000.0, 10.0)


def test_writer_reader_round_trip(T, tmp_path):
    """write_qtf12d (raft/raft_fowt.py:1700-1726, 5 significant digits) -> read_qtf12d."""
    q = T["qtf"]
    p = str(tmp_path / "rt.12d")
    write_qtf12d(p, q, T["w1_2nd"], T["heads_2nd"], float(T["rho"]), float(T["g"]))
    h, w1, w2, q2 = read_qtf12d(p, float(T["rho"]), float(T["g"]))
    np.testing.assert_allclose(w1, T["w1_2nd"], rtol=1e-4)
    np.testing.assert_allclose(q2, q, rtol=1e-4, atol=1e-4 * np.abs(q).max())
