"""Text outputs of the slender-body QTF path (WAMIT .4 / .12d and the f_2nd table).

Formats follow raft/raft_fowt.py:1416-1432 (.4 RAOs), :1700-1726 (.12d QTF) and
:1810-1814 (f_2nd).  Host-side formatting of results already computed on the device.
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
