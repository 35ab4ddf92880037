"""Data-parallel logic on CPU with gloo, world size 2.

* The row-sharded NT-Xent the kernels implement — each rank owns its
  [zj_local; zi_local] rows, all-gathers the projections into the reference's
  global order [zj_all; zi_all] and the per-row lse, and computes the exact
  gradient of its own rows (symmetric W, no column-gradient exchange) —
  reproduces the single-process reference NTXentLoss on the concatenated
  batch, loss and gradients.
* molclr_amd.distributed: init() from the torchrun environment, the flat
  gradient SUM all-reduce and the parameter broadcast.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ntxent_math
from oracle.reference_cpu import RefNTXentLoss

WORLD = 2
B_LOCAL, C, T = 16, 64, 0.1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _inputs():
    rng = np.random.default_rng(0)
    zi = rng.standard_normal((WORLD * B_LOCAL, C)).astype(np.float32)
    zj = (0.5 * zi + rng.standard_normal((WORLD * B_LOCAL, C))).astype(np.float32)
    return zi, zj


def _worker(rank, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(WORLD), LOCAL_RANK=str(rank))
    from molclr_amd import distributed as mdist
    r, w, dev = mdist.init(backend="gloo")
    assert (r, w, dev.type) == (rank, WORLD, "cpu")
    zi, zj = _inputs()
    sl = slice(rank * B_LOCAL, (rank + 1) * B_LOCAL)
    B = WORLD * B_LOCAL
    # local rows [zj_local; zi_local], global indices
    R_local = np.concatenate([zj[sl], zi[sl]], 0)
    rh, nrm = ntxent_math.prep(R_local, True)
    gidx = np.concatenate([np.arange(B_LOCAL) + rank * B_LOCAL,
                           np.arange(B_LOCAL) + rank * B_LOCAL + B])
    # all-gather into [zj_all; zi_all] (two collectives, as ops._NTXent does)
    t = torch.from_numpy(rh)
    cols = torch.empty(2 * B, C, dtype=torch.float64)
    dist.all_gather(list(cols[:B].chunk(WORLD)), t[:B_LOCAL].contiguous())
    dist.all_gather(list(cols[B:].chunk(WORLD)), t[B_LOCAL:].contiguous())
    cols = cols.numpy()
    lse, loss_rows = ntxent_math.rows_forward(rh, gidx, cols, B, T)
    lt = torch.from_numpy(lse)
    lse_cols = torch.empty(2 * B, dtype=torch.float64)
    dist.all_gather(list(lse_cols[:B].chunk(WORLD)), lt[:B_LOCAL].contiguous())
    dist.all_gather(list(lse_cols[B:].chunk(WORLD)), lt[B_LOCAL:].contiguous())
    loss = torch.tensor([loss_rows.sum()])
    dist.all_reduce(loss)
    drh = ntxent_math.rows_backward(rh, gidx, cols, lse_cols.numpy(), B, T)
    dR = ntxent_math.prep_bwd(drh, rh, nrm, True)
    # gradient reduction + broadcast helpers on flat buffers
    flat = torch.full((10,), float(rank + 1))
    mdist.allreduce_grads(flat)
    p = torch.full((4,), float(rank))
    mdist.broadcast_params(p)
    out_q.put((rank, float(loss.item()), dR[B_LOCAL:], dR[:B_LOCAL], flat.tolist(), p.tolist()))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_ntxent_matches_single_process_reference():
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(WORLD)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    zi, zj = _inputs()
    a = torch.from_numpy(zi).requires_grad_(True)
    b = torch.from_numpy(zj).requires_grad_(True)
    ref = RefNTXentLoss("cpu", WORLD * B_LOCAL, T, True)(a, b)
    ref.backward()
    dzi = np.concatenate([r[2] for r in res], 0)
    dzj = np.concatenate([r[3] for r in res], 0)
    for r in res:
        assert abs(r[1] - ref.item()) < 1e-5 * ref.item()
        assert r[4] == [3.0] * 10        # SUM over ranks 1 + 2
        assert r[5] == [0.0] * 4         # rank 0's values broadcast
    assert np.linalg.norm(dzi - a.grad.numpy()) <= 1e-5 * np.linalg.norm(a.grad.numpy())
    assert np.linalg.norm(dzj - b.grad.numpy()) <= 1e-5 * np.linalg.norm(b.grad.numpy())
