"""Time the READ-ONLY reference's Model.solveDynamics on one C2 golden case (VolturnUS-S,
nw = 1000; the cases of tests/golden/make_golden.py "c2"), one core, and print one JSON line.
Build container only (the reference is not on the GPU box); run by tools/calibrate_cpu.py
--interleave with the reference environment of make_golden.py:

    PYTHONPATH=tests/golden/refshim:/root/reference:tests/golden OPENBLAS_NUM_THREADS=1 \
        python tools/ref_time_c2.py CASE
"""
import json
import os
import sys

import make_golden as G   # tests/golden/make_golden.py (imports the reference as `raft`)


def main(ic):
    design = G.load_design(os.path.join(G.REF, "examples", "VolturnUS-S_example.yaml"), min_freq=0.0002)
    case = dict(G.seeded_cases(4, 20241017)[ic])
    model = G.raft.Model(design)
    fowt = model.fowtList[0]
    G.prepare_fowt(fowt, case)
    _, iters, conv, dt = G.run_solve(model, case)
    print(json.dumps({"case": ic, "reference_s": dt, "iters": iters, "conv": conv}))


if __name__ == "__main__":
    main(int(sys.argv[1]))
