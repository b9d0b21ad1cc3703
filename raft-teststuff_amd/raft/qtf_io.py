"""WAMIT-format QTF files and the text outputs of the second-order path.

Formats follow raft/raft_fowt.py:1416-1432 (.4 RAOs), :1651-1697 (.12d reader),
:1700-1726 (.12d writer) and :1810-1814 (f_2nd).  Host-side parsing / formatting of data
that the device kernels consume or produced.
"""
import os

import numpy as np


def qtf_file_names(folder, beta, iCase=None, iWT=None):
    whead = f"{np.degrees(beta) % 360:.2f}".replace(".", "p")
    if isinstance(iCase, int) and isinstance(iWT, int):
        tag = f"_Head{whead}_Case{iCase + 1}_WT{iWT}"
    else:
        tag = f"_Head{whead}"
    return (os.path.join(folder, f"raos-slender_body{tag}.4"),
            os.path.join(folder, f"qtf-slender_body-total{tag}.12d"))


def write_rao4(path, w1, beta, Xi):
    """Columns: period, heading (as given, rad), DoF, |x|, phase, Re, Im."""
    with open(path, "w") as f:
        for iDoF in range(Xi.shape[0]):
            for w, x in zip(w1, Xi[iDoF]):
                f.write(f"{2 * np.pi / w: 8.4e} {beta: 8.4e} {iDoF + 1} {np.abs(x): 8.4e} {np.angle(x): 8.4e} "
                        f"{x.real: 8.4e} {x.imag: 8.4e}\n")


def write_qtf12d(path, qtf, w1, heads, rho, g, ULEN=1):
    """Upper triangle of qtf [n1, n2, nh, 6] scaled by 1/(rho g ULEN)."""
    n1 = len(w1)
    iu, ju = np.triu_indices(n1)
    with open(path, "w") as f:
        for ih in range(len(heads)):
            hd = np.rad2deg(heads[ih])
            for iDoF in range(qtf.shape[3]):
                F = qtf[iu, ju, ih, iDoF] / (rho * g * ULEN)
                for a, b, x in zip(iu, ju, F):
                    f.write(f"{2 * np.pi / w1[a]: 8.4e} {2 * np.pi / w1[b]: 8.4e} {hd: 8.4e} {hd: 8.4e} {iDoF + 1} "
                            f"{np.abs(x): 8.4e} {np.angle(x): 8.4e} {x.real: 8.4e} {x.imag: 8.4e}\n")


def write_f2nd(path, w, f):
    with open(path, "w") as fh:
        for wi, row in zip(w, f.T):
            fh.write(f"{wi:.5f} {row[0]:.5f} {row[1]:.5f} {row[2]:.5f} {row[3]:.5f} {row[4]:.5f} {row[5]:.5f}\n")


def read_qtf12d(src, rho, g, ULEN=1, nDOF=6):
    """FOWT.readQTF (raft/raft_fowt.py:1651-1697): a WAMIT .12d file (path, or its numeric
    table as loaded by np.loadtxt) -> (heads_2nd [rad], w1_2nd, w2_2nd, qtf [n1, n2, nh, 6]).

    Columns: period 1, period 2, heading 1, heading 2 [deg], DoF (1-6), |F|, phase, Re, Im.
    Same results as the reference's row loop: frequencies 2 pi / period and headings are
    matched exactly against their sorted unique values, entries are scaled by rho g ULEN
    (rho g ULEN^2 for moments), and each row also writes the conjugate at the mirrored
    position (Hermitian fill); rows are applied in file order, so a later row wins."""
    data = np.array(np.loadtxt(src) if isinstance(src, (str, os.PathLike)) else src, dtype=float, copy=True)
    data = np.atleast_2d(data)
    data[:, 0:2] = 2.0 * np.pi / data[:, 0:2]
    if not (data[:, 2] == data[:, 3]).all():
        raise ValueError("Only unidirectional QTFs are supported for now.")
    heads = np.deg2rad(np.sort(np.unique(data[:, 2])))
    w1 = np.unique(data[:, 0])
    w2 = np.unique(data[:, 1])
    if len(w1) != len(w2) or not (w1 == w2).all():
        raise ValueError("Both frequency columns in the input QTF must contain the same values.")
    i1 = np.searchsorted(w1, data[:, 0])
    i2 = np.searchsorted(w2, data[:, 1])
    # The reference looks a row's heading up as np.where(heads_2nd == row[2]) (:1686): the
    # heading column in DEGREES against heads_2nd in RADIANS.  Heading 0 matches; a heading
    # with no radian value equal to its degree value finds nothing and indhead[0] raises
    # IndexError.  Mirrored exactly, error included.
    ih = np.minimum(np.searchsorted(heads, data[:, 2]), len(heads) - 1)
    miss = heads[ih] != data[:, 2]
    if miss.any():
        raise IndexError("index 0 is out of bounds for axis 0 with size 0 (readQTF matches the .12d heading "
                         f"{data[np.argmax(miss), 2]} deg against headings in radians, raft/raft_fowt.py:1686)")
    idof = np.round(data[:, 4] - 1).astype(int)
    factor = np.where(idof >= 3, rho * g * ULEN * ULEN, rho * g * ULEN)
    val = factor * (data[:, 7] + 1j * data[:, 8])
    # sequential semantics: row r writes (i1, i2) = v, then (i2, i1) = conj(v) off the diagonal
    n = len(data)
    off = i1 != i2
    rows = np.concatenate([np.arange(n), np.nonzero(off)[0]])
    order = np.concatenate([2 * np.arange(n), 2 * np.nonzero(off)[0] + 1])
    a = np.concatenate([i1, i2[off]])
    b = np.concatenate([i2, i1[off]])
    v = np.concatenate([val, np.conj(val[off])])
    qtf = np.zeros([len(w1), len(w2), len(heads), nDOF], dtype=complex)
    key = ((a * len(w2) + b) * len(heads) + ih[rows]) * nDOF + idof[rows]
    last = np.lexsort((order, key))            # per key, the highest write order comes last
    keep = np.ones(len(key), dtype=bool)
    ks = key[last]
    keep[:-1] = ks[1:] != ks[:-1]
    sel = last[keep]
    qtf.reshape(-1)[key[sel]] = v[sel]
    return heads, w1, w2, qtf
