"""Host preparation of a design sweep in worker processes (raft/batch.py host_pool,
prepare_design): the models that come back are identical to the serial path, including the
all-zero per-bin matrices that travel as shape tags (raft/fowt.py _Zeros)."""
import json
import os

import numpy as np

import raft  # noqa: F401
from raft import Model
from raft.batch import host_pool, prepare_design
from raft.sweep import sweep_multipliers, sweep_variant

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _state(m):
    f = m.fowtList[0]
    out = {k: v for k, v in f.__dict__.items() if isinstance(v, np.ndarray)}
    for i, mem in enumerate(f.memberList):
        out.update({f"m{i}.{k}": v for k, v in mem.__dict__.items() if isinstance(v, np.ndarray)})
    return out


def test_pool_matches_serial():
    with open(os.path.join(ROOT, "tests", "golden", "designs", "VolturnUS-S_example.json")) as fh:
        base = json.load(fh)
    base["settings"]["min_freq"] = 0.005
    C_moor = np.load(os.path.join(ROOT, "tests", "golden", "c2_nw1000.npz"))["C_moor"]
    mult = sweep_multipliers(3)
    jobs = [(sweep_variant(base, mult[i]), {"C_moor": C_moor}, None, 0) for i in range(3)]
    serial = [prepare_design(j) for j in jobs]
    grid = (Model.frequency_grid(base), float(base["site"]["water_depth"]))
    pool = host_pool(2, grids=[grid])
    try:
        pooled = pool.map(prepare_design, jobs, chunksize=1)
    finally:
        pool.close()
        pool.join()
    for a, b in zip(serial, pooled):
        sa, sb = _state(a), _state(b)
        assert sa.keys() == sb.keys()
        for k in sa:
            np.testing.assert_array_equal(sa[k], sb[k], err_msg=k)
        assert b.fowtList[0]._dd is None
        assert np.all(b.fowtList[0].A_BEM == 0) and b.fowtList[0].A_BEM.shape == a.fowtList[0].A_BEM.shape


def test_light_designs_carry_the_device_tables():
    """DesignBatch(light=True) ships HostDesign records: the same device tables and scalars
    as the full prepared model, far smaller when pickled."""
    import pickle
    with open(os.path.join(ROOT, "tests", "golden", "designs", "VolturnUS-S_example.json")) as fh:
        base = json.load(fh)
    base["settings"]["min_freq"] = 0.005
    C_moor = np.load(os.path.join(ROOT, "tests", "golden", "c2_nw1000.npz"))["C_moor"]
    full = prepare_design((base, {"C_moor": C_moor}, None, 0))
    light = pickle.loads(pickle.dumps(prepare_design((base, {"C_moor": C_moor}, None, 0, True))))
    a, b = full.fowtList[0].host_tables(), light.host_tables()
    np.testing.assert_array_equal(a["packed"], b["packed"])
    np.testing.assert_array_equal(a["mstart"], b["mstart"])
    assert a["layout"] == b["layout"] and (a["nn"], a["nm"], a["per_bin"]) == (b["nn"], b["nm"], b["per_bin"])
    f = full.fowtList[0]
    assert (light.nw, light.dw, light.depth, light.rho_water, light.g) == (f.nw, f.dw, f.depth, f.rho_water, f.g)
    assert (light.nIter, light.XiStart) == (full.nIter, full.XiStart)
    np.testing.assert_array_equal(light.w, full.w)
    assert len(pickle.dumps(light)) < len(pickle.dumps(full)) / 2
