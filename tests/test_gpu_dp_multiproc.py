"""The data-parallel product path with two real ranks on the GPU.

Two processes share the box's GPU over the gloo backend (RCCL wants one GPU
per rank; gloo runs the same torch.distributed calls on the same CUDA
tensors), so the multi-rank code paths -- row-sharded NT-Xent with its
all-gathers, the overlapped bucketed gradient all-reduce driven by the
executor's events, FusedAdam, bench.py's world > 1 branch and its
max-over-ranks timing -- run end to end here, not only under gloo on CPU.
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _torchrun(args, timeout):
    env = dict(os.environ, MOLCLR_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), *args]
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


def test_dp_step_two_ranks():
    r = _torchrun([str(ROOT / "tools" / "dp_check.py")], 240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "DP_OK world=2" in r.stdout, r.stdout[-2000:]


def test_bench_two_ranks():
    r = _torchrun([str(ROOT / "bench.py"), "--gpus", "2", "--config", "c1", "--steps", "4",
                   "--warmup", "2", "--batches", "2", "--no-cpu-baseline", "--mfma-steps", "1"], 240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints the one JSON line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 4 and out["value"] > 0
    assert out["config"]["global_batch"] == 128 and out["scaling"] == "weak"
