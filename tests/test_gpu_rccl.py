"""RCCL on the GPU: torch.distributed backend "nccl" (RCCL on ROCm) at world size 1 on this
box's one MI355X.  A child process initialises the group before any other GPU work and runs
the three exchanges of raft/parallel.py through it -- the all-gather of a case-sharded batch's
outputs (gather_cases), the packed-pair all-gather of the tile-sharded QTF (assemble_qtf) and
the per-iteration all-reduces of the bin-sharded drag fixed point (solve_bins_sharded); this
process runs the same workloads without a process group.  The results must be equal bit for
bit: the exchanges move and add exact copies (x + 0 == x), whatever the backend.  More ranks
than GPUs are not simulated; N > 1 is covered by the gloo tests (tests/test_parallel.py)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

HERE = os.path.dirname(os.path.abspath(__file__))
pytestmark = pytest.mark.gpu


def test_rccl_world1_exchanges_equal_single_device(tmp_path):
    sys.path.insert(0, os.path.join(HERE, "helpers"))
    from rccl_cases import run_all
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    out = tmp_path / "rccl.npz"
    p = subprocess.run([sys.executable, os.path.join(HERE, "helpers", "rccl_world1.py"), str(out)], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    got = dict(np.load(out))
    assert str(got.pop("backend")) == "nccl"
    ref = run_all(group=None)
    assert set(got) == set(ref)
    for k in ref:
        np.testing.assert_array_equal(got[k], np.asarray(ref[k]), err_msg=k)
