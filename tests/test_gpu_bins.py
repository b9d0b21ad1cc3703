"""GPU parity of the bin-sharded drag fixed point (SURVEY.md §8(e) row 2:
rh_lin_partial_sums / rh_bin_step through the C-ABI, driven by
raft/parallel.py solve_bins_sharded).  One device, so the bin split is exercised with
several shards owned by this process (their partial sums are combined exactly as the
all-reduce over ranks combines them); the collective skeleton itself is covered by the
gloo world-2 test in tests/test_parallel.py.  Against the reference goldens: Xi within
1e-9 relative, identical drag-iteration counts."""
import numpy as np
import pytest

from conftest import golden_cases, load_golden
from test_gpu_parity import make_model, rel

pytestmark = pytest.mark.gpu
RTOL = 1e-9


@pytest.mark.parametrize("tag,design,settings", [("c1_OC3spar", "OC3spar", None),
                                                 ("c2_nw200", "VolturnUS-S_example", None)])
@pytest.mark.parametrize("nshard", [1, 2, 5])
def test_bin_sharded_solve_matches_reference(tag, design, settings, nshard):
    from raft.parallel import bin_shard, solve_bins_sharded
    T = load_golden(tag)
    m, f = make_model(design, T, settings)
    shards = [bin_shard(m.nw, r, nshard) for r in range(nshard)]
    for ic, case in enumerate(golden_cases(T)):
        Xi, iters, status, B = solve_bins_sharded(f, case, m.nIter, m.XiStart, shards=shards)
        assert iters == int(T["out_iters"][ic]), (ic, iters, int(T["out_iters"][ic]))
        assert (status == 1) == bool(T["out_conv"][ic])
        assert rel(Xi, T["out_Xi"][ic][0]) < RTOL, (ic, rel(Xi, T["out_Xi"][ic][0]))
        assert rel(B, T["out_B_drag"][ic]) < RTOL


def test_bin_sharded_nan_raises_reference_message():
    from raft.parallel import solve_bins_sharded
    T = load_golden("c1_OC3spar")
    m, f = make_model("OC3spar", T)
    case = dict(wave_spectrum="JONSWAP", wave_period=10, wave_height=float("nan"), wave_heading=0)
    with pytest.raises(Exception, match="Nan detected in response vector Xi."):
        solve_bins_sharded(f, case, m.nIter, m.XiStart, shards=[(0, 40), (40, m.nw)])
