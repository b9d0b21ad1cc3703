"""Child process of tests/test_gpu_rccl.py: torch.distributed with backend "nccl" (RCCL on
ROCm) at world size 1, initialised before any other GPU work in this process; then the three
exchanges of raft/parallel.py run through it (gather_cases, assemble_qtf, solve_bins_sharded)
and their results are saved for the parent to compare with the single-device path.

usage: python rccl_world1.py OUT.npz   (env: MASTER_ADDR, MASTER_PORT; RANK=0, WORLD_SIZE=1)"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))           # tests/ (conftest helpers)


def main(out):
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    from rccl_cases import run_all
    res = run_all(group=dist.group.WORLD)
    res["backend"] = np.array(dist.get_backend())
    np.savez(out, **res)
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
