"""Repeat tests/test_gpu_graph_step.py::test_capacity_fit_lookup_and_prepare
in one process and report which repetitions fail (an intermittent failure
shows up as zero MLP weight gradients on the captured side).

    python tools/cf_stress.py [reps]
"""
import sys
import traceback
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from tests import test_gpu_graph_step as t  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    fails = 0
    if "--keep" in sys.argv:  # keep every model alive: no id / address reuse across reps
        keep = []
        orig = t._make

        def make(kind, seed):
            m = orig(kind, seed)
            keep.append(m)
            return m
        t._make = make
    import gc
    for i in range(reps):
        if "--gc" in sys.argv:
            gc.collect()
            torch.cuda.synchronize()
        try:
            t.test_capacity_fit_lookup_and_prepare(dev)
            print(f"rep {i}: ok", flush=True)
        except AssertionError as e:
            fails += 1
            print(f"rep {i}: FAIL {str(e)[:400]}", flush=True)
        except Exception:  # noqa: BLE001
            traceback.print_exc()
            raise
    print(f"{fails} of {reps} failed", flush=True)


if __name__ == "__main__":
    main()
