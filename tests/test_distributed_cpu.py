"""Data-parallel logic on CPU with gloo, world size 2.

* The row-sharded NT-Xent the kernels implement — each rank owns its
  [zj_local; zi_local] rows, all-gathers the projections into the reference's
  global order [zj_all; zi_all] and the per-row lse, and computes the exact
  gradient of its own rows (symmetric W, no column-gradient exchange) —
  reproduces the single-process reference NTXentLoss on the concatenated
  batch, loss and gradients.
* The product's exchange helpers (molclr_amd.distributed.gather_rows /
  gather_lse / global_row_index, what ops._NTXent calls) produce the
  reference's global order.
* molclr_amd.distributed: init() from the torchrun environment, the flat
  gradient SUM all-reduce and the parameter broadcast.
* Data parallel input: MoleculeDatasetWrapper gives each rank a disjoint,
  equally sized shard, reshuffled every epoch (identical per-rank
  data made every row meet copies of itself as negatives).
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
    # the product's exchange (molclr_amd.distributed, as ops._NTXent calls it):
    # one gather of [zj_local; zi_local] into [zj_all; zi_all], global row ids
    gidx = mdist.global_row_index(B_LOCAL, rank, WORLD, "cpu").numpy().astype(np.int64)
    assert np.array_equal(gidx, np.concatenate([np.arange(B_LOCAL) + rank * B_LOCAL,
                                                np.arange(B_LOCAL) + rank * B_LOCAL + B]))
    cols = mdist.gather_rows(torch.from_numpy(rh)).numpy()
    Rall = np.concatenate([zj, zi], 0)
    assert np.allclose(cols, ntxent_math.prep(Rall, True)[0])
    lse, loss_rows = ntxent_math.rows_forward(rh, gidx, cols, B, T)
    lse_cols = mdist.gather_lse(torch.from_numpy(lse)).numpy()
    assert np.allclose(lse_cols, ntxent_math.rows_forward(cols, np.arange(2 * B), cols, B, T)[0])
    loss = torch.tensor([loss_rows.sum()])
    dist.all_reduce(loss)
    drh = ntxent_math.rows_backward(rh, gidx, cols, lse_cols, B, T)
    dR = ntxent_math.prep_bwd(drh, rh, nrm, True)
    # data sharding: disjoint, equally sized per-rank shards every epoch
    from molclr_amd.dataset import MoleculeDatasetWrapper
    w = MoleculeDatasetWrapper(8, 0, 0.2, "synthetic:120", seed=3)
    tr, va = w.get_data_loaders()
    ids = []
    for epoch in range(2):
        ids.append(list(tr.sampler))
    first = next(iter(tr))[0]
    nb = torch.tensor([len(tr), len(va)])
    nbs = [torch.zeros(2, dtype=torch.long) for _ in range(WORLD)]
    dist.all_gather(nbs, nb)
    shard = torch.tensor(sorted(ids[0]))
    shards = [torch.zeros_like(shard) for _ in range(WORLD)]
    dist.all_gather(shards, shard)
    xs = torch.tensor([first.x.shape[0]])
    sizes = [torch.zeros_like(xs) for _ in range(WORLD)]
    dist.all_gather(sizes, xs)
    sharding = ([n.tolist() for n in nbs], [s.tolist() for s in shards], ids[0] != ids[1])
    # gradient reduction + broadcast helpers on flat buffers
    flat = torch.full((10,), float(rank + 1))
    mdist.allreduce_grads(flat)
    p = torch.full((4,), float(rank))
    mdist.broadcast_params(p)
    out_q.put((rank, float(loss.item()), dR[B_LOCAL:], dR[:B_LOCAL], flat.tolist(), p.tolist(),
               sharding))
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
    nbs, shards, reshuffled = res[0][6]
    assert nbs[0] == nbs[1] and nbs[0][0] > 0       # equal batch counts per rank
    assert not set(shards[0]) & set(shards[1])      # disjoint molecule shards
    assert reshuffled                                 # a new permutation every epoch
    assert np.linalg.norm(dzi - a.grad.numpy()) <= 1e-5 * np.linalg.norm(a.grad.numpy())
    assert np.linalg.norm(dzj - b.grad.numpy()) <= 1e-5 * np.linalg.norm(b.grad.numpy())
