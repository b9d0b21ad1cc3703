"""Extract the reference's OWN statics golden values into a data fixture.

Reads, as text, the expected values that the reference's tests hold
(tests/test_member.py `desired_*` lists for ten single-member designs, tests/test_fowt.py
`desired_*` lists for VolturnUS-S and OC3spar) and the ten member input files of
tests/test_data/, and writes them as plain data to tests/golden/statics_ref.npz and
tests/golden/statics_members.json.  Only literal numbers and input dictionaries are
written; no reference source text.  Runs in the build container only:

    python tests/golden/make_statics_golden.py
"""
import ast
import json
import os

import numpy as np
import yaml

REF = "/root/reference/tests"
HERE = os.path.dirname(os.path.abspath(__file__))
MEMBER_FILES = ["mem_srf_vert_circ_cyl.yaml", "mem_srf_vert_rect_cyl.yaml", "mem_srf_pitch_circ_cyl.yaml",
                "mem_srf_pitch_rect_cyl.yaml", "mem_srf_inc_circ_cyl.yaml", "mem_srf_inc_rect_cyl.yaml",
                "mem_subm_horz_circ_cyl.yaml", "mem_subm_horz_rect_cyl.yaml", "mem_srf_vert_tap_circ_cyl.yaml",
                "mem_srf_vert_tap_rect_cyl.yaml"]   # order of tests/test_member.py:22-33


def desired_values(path):
    """Every module-level `desired_<name> = <literal list>` of a test file, evaluated as
    data (list / np.array literals only)."""
    tree = ast.parse(open(path).read())
    out = {}
    for node in tree.body:
        if isinstance(node, ast.Assign) and len(node.targets) == 1 and isinstance(node.targets[0], ast.Name):
            name = node.targets[0].id
            if name.startswith("desired_"):
                expr = compile(ast.Expression(node.value), path, "eval")
                out[name[len("desired_"):]] = eval(expr, {"__builtins__": {}, "np": np})
    return out


def main():
    arrays = {}
    for k, v in desired_values(os.path.join(REF, "test_member.py")).items():
        arrays["member_" + k] = np.array([np.asarray(x, dtype=float) for x in v])
    for k, v in desired_values(os.path.join(REF, "test_fowt.py")).items():
        if np.iscomplexobj(np.asarray(v[0])):
            continue            # excitation goldens: not statics values
        for i, x in enumerate(v):   # per design: some entries (m_ballast) are ragged across designs
            arrays[f"fowt_{k}_{i}"] = np.asarray(x, dtype=float)
    np.savez(os.path.join(HERE, "statics_ref.npz"), **arrays)
    members = []
    for f in MEMBER_FILES:
        with open(os.path.join(REF, "test_data", f)) as fh:
            members.append(yaml.safe_load(fh))
    with open(os.path.join(HERE, "statics_members.json"), "w") as fh:
        json.dump(members, fh, indent=1)
    print({k: v.shape for k, v in arrays.items()})


if __name__ == "__main__":
    main()
