"""Repeat tests/test_gpu_dp.py::test_captured_dp_step_rccl_world1 under one
RCCL world-1 process group and report which repetitions fail.

    python tools/dp_stress.py [reps] [--gc]
"""
import gc
import os
import socket
import sys
from pathlib import Path

import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from tests import test_gpu_dp as t  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device("cuda", 0)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    fails = 0
    try:
        for i in range(reps):
            if "--gc" in sys.argv:
                gc.collect()
            for kind in ("gin", "gcn"):
                try:
                    t.test_captured_dp_step_rccl_world1(dev, dist.group.WORLD, kind)
                    print(f"rep {i} {kind}: ok", flush=True)
                except AssertionError as e:
                    fails += 1
                    print(f"rep {i} {kind}: FAIL {str(e)[:200]}", flush=True)
    finally:
        dist.destroy_process_group()
    print(f"{fails} of {2 * reps} failed", flush=True)


if __name__ == "__main__":
    main()
