"""Design x sea-state sweeps (BASELINE.json configs[4]).

The reference sweeps VolturnUS-S geometry with five variables, nested loops over
{0.75, 1, 1.25} x baseline (raft/parametersweep.py:33-47) and one runRAFT per design
(:91).  The C5 workload draws the same five multipliers from U(0.75, 1.25) and pairs every
design with a fixed sea-state grid.  A sweep here is then:
  * per design: host preparation (members, statics, added mass; raft/statics.py,
    raft/member.py) and the device wave tables (rh_wave_tables), once per (design, heading);
  * one rh_solve_cases launch over every (design, sea state) case of the batch.

This module imports only numpy: tests/golden/make_golden.py loads it by file path to build
the very same variants for the reference run.
"""
import copy

import numpy as np

SWEEP_VARIABLES = ("ccD", "ocD", "T", "ocR", "pH")   # raft/parametersweep.py:33-37


def sweep_baseline(design):
    """The five swept quantities of a VolturnUS-S-style platform (raft/parametersweep.py:33-37):
    centre-column diameter, outer-column diameter, draft (rA z of the centre column, negative),
    outer-column radius, pontoon height."""
    m = design["platform"]["members"]
    T = m[0]["rA"][2]
    return dict(ccD=float(m[0]["d"]), ocD=float(m[1]["d"]), T=float(T), ocR=float(m[1]["rA"][0]),
                pH=float((m[2]["rA"][2] - T) * 2))


def sweep_variant(design, mult):
    """A copy of `design` with the five variables scaled by `mult` (5 factors, order of
    SWEEP_VARIABLES).  The member edits restate the assignments of the reference's nested
    loops (raft/parametersweep.py:56-88) in the same order, applied once to the baseline:
    the reference mutates one design cumulatively across loop iterations, which only
    matters for its 3-level grid, not for an independent draw.  Mooring point moves
    (:62-66, :78-83) are skipped: the mooring stiffness is an input here."""
    d = copy.deepcopy(design)
    d["platform"]["members"][:4] = variant_members(design, mult)
    return d


def variant_members(design, mult):
    """The four platform members sweep_variant edits (copies, in member order), with its
    assignments applied; everything else of the variant is the base design."""
    base = sweep_baseline(design)
    a, b, c, dd, e = (base[k] * float(f) for k, f in zip(SWEEP_VARIABLES, mult))
    # shallow copies suffice: every list edited below (rA, rB, the pontoon's d) is replaced by
    # a fresh list before it is written
    m = [dict(mm) for mm in design["platform"]["members"][:4]]
    for mm in m[:4]:
        mm["rA"] = [float(x) for x in mm["rA"]]
        mm["rB"] = [float(x) for x in mm["rB"]]
    m[2]["d"] = [float(x) for x in m[2]["d"]]
    # centre-column diameter (:56-58)
    m[0]["d"] = a
    m[2]["rA"][0] = m[2]["rA"][0] * (a / base["ccD"])
    m[3]["rA"][0] = m[3]["rA"][0] * (a / base["ccD"])
    # outer-column diameter (:60-62)
    m[1]["d"] = b
    m[2]["rB"][0] = m[1]["rA"][0] - b / 2
    m[3]["rB"][0] = m[1]["rB"][0] - b / 2
    # draft (:68-72)
    m[0]["rA"][2] = c
    m[1]["rA"][2] = c
    m[2]["rA"][2] = c + m[2]["d"][1] / 2
    m[2]["rB"][2] = c + m[2]["d"][1] / 2
    # outer-column radius (:74-78)
    m[1]["rA"][0] = dd
    m[1]["rB"][0] = dd
    m[2]["rB"][0] = dd - m[1]["d"] / 2
    m[3]["rB"][0] = dd - m[1]["d"] / 2
    # pontoon height (:85-87)
    m[2]["d"][1] = e
    m[2]["rA"][2] = m[0]["rA"][2] + e / 2
    m[2]["rB"][2] = m[1]["rA"][2] + e / 2
    return m


def sweep_multipliers(n_designs, seed=20241016, lower=0.75, upper=1.25):
    """C5 design draws: U(lower, upper) per variable."""
    rng = np.random.default_rng(seed)
    return rng.uniform(lower, upper, size=(n_designs, len(SWEEP_VARIABLES)))


def sea_state_grid(Hs=(2, 4, 6, 8, 10), Tp=tuple(range(6, 22, 2)), heading=0.0, gamma=0.0):
    """C5 sea states: Hs x Tp (40 by default), heading 0, IEC automatic gamma."""
    return [dict(wave_spectrum="JONSWAP", wave_height=float(h), wave_period=float(t), wave_heading=float(heading),
                 wave_gamma=float(gamma)) for h in Hs for t in Tp]
