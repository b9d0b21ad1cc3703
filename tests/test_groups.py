"""Host logic of the lock-step case groups (rh_cases.group_start, raft/solver.py)."""
import numpy as np

import raft  # noqa: F401  (puts the package on the path via conftest)
from raft.solver import case_groups


def test_groups_break_on_design_heading_and_width():
    design = np.array([0, 0, 0, 0, 0, 1, 1, 1])
    head = np.array([0, 0, 0, 1, 1, 0, 0, 0])
    g = case_groups(design, head, 2)
    assert g.tolist() == [0, 2, 3, 5, 7, 8]
    for a, b in zip(g[:-1], g[1:]):
        assert 1 <= b - a <= 2
        assert len(set(design[a:b])) == 1 and len(set(head[a:b])) == 1


def test_groups_edge_sizes():
    assert case_groups(np.zeros(0, int), np.zeros(0, int), 2).tolist() == [0]
    assert case_groups(np.zeros(1, int), np.zeros(1, int), 2).tolist() == [0, 1]
    assert case_groups(np.zeros(5, int), np.zeros(5, int), 1).tolist() == [0, 1, 2, 3, 4, 5]
    assert case_groups(np.zeros(5, int), np.zeros(5, int), 4).tolist() == [0, 4, 5]
