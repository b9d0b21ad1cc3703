"""CPU: the C-ABI library builds for gfx950, loads, and exports every entry point that
include/rafthip.h declares (no compute calls -- there is no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "rafthip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|long long|const char\*)\s+(rh_\w+)\s*\(", src, flags=re.M)))


@pytest.fixture(scope="module")
def libpath():
    import __graft_entry__ as g
    g.build()
    return g.LIB


def test_header_declares_the_boundary():
    fns = declared_functions()
    for must in ["rh_ctx_create", "rh_ctx_destroy", "rh_last_error", "rh_wave_tables", "rh_solve_cases",
                 "rh_heading_response", "rh_linearize", "rh_drag_excitation", "rh_sea_state", "rh_motion_stats",
                 "rh_system_solve", "rh_version", "rh_qtf_workspace_bytes", "rh_qtf_slender", "rh_force_2nd",
                 "rh_force_2nd_spectrum"]:
        assert must in fns


def test_library_exports_every_declared_symbol(libpath):
    out = subprocess.run(["nm", "-D", "--defined-only", libpath], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\sT\s(rh_\w+)$", out, flags=re.M))
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing


def test_library_loads_and_binds(libpath):
    from raft import _native as N
    L = N.lib()
    assert L.rh_version() == 7
    assert L.rh_group_cases() >= 1
    # the tuning knobs live on a context (no mutable process globals);
    # without a GPU there is no context, and a null one is rejected
    assert L.rh_set_solver(None, 0) == N.RH_EINVAL
    assert L.rh_set_qtf_waves(None, 4) == N.RH_EINVAL
    assert b"null context" in L.rh_last_error()
    for f in declared_functions():
        assert hasattr(L, f)


def test_library_is_gfx950(libpath):
    """The embedded code object targets gfx950 (MI355X) only."""
    data = open(libpath, "rb").read()
    assert b"gfx950" in data
    for other in (b"gfx90a", b"gfx942", b"gfx1100"):
        assert other not in data


def test_struct_layout_matches_header():
    """ctypes mirrors must match the C structs (field count / order by name)."""
    from raft import _native as N
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)

    def fields(name):
        body = re.search(r"typedef struct \{([^{}]*)\}\s*" + name + ";", src).group(1)
        names = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            names += [n.strip().lstrip("*") for n in decl.split(" ", 1)[1].replace("*", " ").split(",")]
        return [n.split()[-1] for n in names]

    assert fields("rh_design") == [f[0] for f in N.RhDesign._fields_]
    assert fields("rh_cases") == [f[0] for f in N.RhCases._fields_]
    assert fields("rh_solve_out") == [f[0] for f in N.RhSolveOut._fields_]
    assert fields("rh_qtf_design") == [f[0] for f in N.RhQtfDesign._fields_]


def test_product_fails_loudly_without_gpu():
    """No CPU fallback: device paths raise when no GPU is visible."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    import raft
    from conftest import load_design, load_golden, statics_of
    T = load_golden("c1_OC3spar")
    m = raft.Model(load_design("OC3spar"), statics=[statics_of(T)])
    f = m.fowtList[0]
    f.setPosition(T["r6"])
    f.calcStatics()
    f.calcHydroConstants()
    with pytest.raises(Exception):
        m.solveDynamics({"wave_heading": 0, "wave_period": 10, "wave_height": 2})
