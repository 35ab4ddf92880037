"""Host-side logic: synthetic generator, node-mask augmentation (dataset.py:111-145
semantics), collate (PyG 1.6.3), and the oracle graph build."""
import math

import numpy as np
import torch

from molclr_amd.data import Batch, Data
from molclr_amd.dataset import (MASK_ATOM, MoleculeDataset, SyntheticPairBatches, collate_views,
                                mask_view, random_molecule)
from oracle.graph_ref import graph_build


def test_molecule_layout():
    rng = np.random.default_rng(0)
    for _ in range(50):
        m = random_molecule(rng)
        N, M = m.num_atoms, m.num_bonds
        assert 10 <= N <= 50
        assert M == (N - 1) + N // 8
        ei, ea = m.edge_index, m.edge_attr
        # consecutive (s,e),(e,s) pairs with identical attributes (dataset.py:93-109)
        assert np.array_equal(ei[0, 0::2], ei[1, 1::2]) and np.array_equal(ei[1, 0::2], ei[0, 1::2])
        assert np.array_equal(ea[0::2], ea[1::2])
        assert ea[:, 0].max() <= 3 and ea[:, 1].max() <= 2
        assert m.x[:, 0].max() < 118 and m.x[:, 1].max() <= 2
        # connected: recursive tree
        seen = {0}
        adj = {i: set() for i in range(N)}
        for s, e in ei.T:
            adj[int(s)].add(int(e))
        stack = [0]
        while stack:
            u = stack.pop()
            for v in adj[u]:
                if v not in seen:
                    seen.add(v)
                    stack.append(v)
        assert len(seen) == N


def test_pubchem_shape_bounds():
    rng = np.random.default_rng(1)
    ns = [random_molecule(rng, "pubchem").num_atoms for _ in range(300)]
    assert min(ns) >= 6 and max(ns) <= 80 and 22 < np.mean(ns) < 32


def test_mask_view_semantics():
    rng = np.random.default_rng(2)
    m = random_molecule(rng)
    N, M = m.num_atoms, m.num_bonds
    x, ei, ea = mask_view(m, np.random.default_rng(3))
    nm = max(1, math.floor(0.25 * N))
    ne = max(0, math.floor(0.25 * M))
    assert (x[:, 0] == MASK_ATOM).sum() >= nm - (m.x[:, 0] == MASK_ATOM).sum()
    assert ((x != m.x).any(1)).sum() <= nm
    assert ((x == [MASK_ATOM, 0]).all(1)).sum() == nm
    assert ei.shape[1] == 2 * (M - ne) and ea.shape[0] == 2 * (M - ne)
    # survivors keep original order and stay paired
    orig = [tuple(c) for c in m.edge_index.T]
    pos = [orig.index(tuple(c)) for c in ei.T]
    assert pos == sorted(pos)
    assert all(pos[2 * k] % 2 == 0 and pos[2 * k + 1] == pos[2 * k] + 1 for k in range(len(pos) // 2))


def test_views_are_independent_and_reproducible():
    a = SyntheticPairBatches(8, seed=0).next()
    b = SyntheticPairBatches(8, seed=0).next()
    for u, v in zip(a, b):
        assert torch.equal(u.x, v.x) and torch.equal(u.edge_index, v.edge_index)
    assert not torch.equal(a[0].x, a[1].x)


def test_collate_matches_from_data_list():
    rng = np.random.default_rng(4)
    views = [mask_view(random_molecule(rng), rng) for _ in range(5)]
    fast = collate_views(views)
    slow = Batch.from_data_list([Data(x=torch.from_numpy(x), edge_index=torch.from_numpy(ei),
                                      edge_attr=torch.from_numpy(ea)) for x, ei, ea in views])
    for f in ("x", "edge_index", "edge_attr", "batch", "ptr"):
        assert torch.equal(getattr(fast, f), getattr(slow, f)), f
    assert fast.num_graphs == slow.num_graphs == 5


def test_dataset_getitem_contract():
    ds = MoleculeDataset(4, seed=0)
    di, dj = ds[1]
    assert di.x.shape == dj.x.shape and di.x.dtype == torch.long
    assert di.edge_index.shape[0] == 2 and di.edge_attr.shape[1] == 2


def test_oracle_graph_build_properties():
    bi, _ = SyntheticPairBatches(16, seed=5).next()
    N, G = bi.x.shape[0], bi.num_graphs
    g = graph_build(bi.edge_index.numpy(), bi.edge_attr.numpy(), bi.batch.numpy(), N, G)
    ei = bi.edge_index.numpy()
    assert g["rowptr"][-1] == ei.shape[1] and g["rowptr_t"][-1] == ei.shape[1]
    for i in range(N):
        ids = np.nonzero(ei[1] == i)[0]  # edge order
        assert list(g["col"][g["rowptr"][i]:g["rowptr"][i + 1]]) == list(ei[0, ids])
    ec = g["ecount"].reshape(N, 8)
    deg = np.diff(g["rowptr"])
    assert np.array_equal(ec[:, :5].sum(1), deg + 1) and np.array_equal(ec[:, 5:].sum(1), deg + 1)
    assert np.array_equal(g["graph_ptr"], bi.ptr.numpy())
    # neighbour slots: first 4 row entries (+ combined edge type), degree in bits 29..31
    for key, ptr, colk in (("nbr", "rowptr", "col"), ("nbr_t", "rowptr_t", "col_t")):
        slots = g[key].view(np.uint32).reshape(N, 4)
        for i in range(N):
            b, e = g[ptr][i], g[ptr][i + 1]
            assert slots[i, 0] >> 29 == (e - b if e - b <= 4 else 7)
            for s in range(min(4, e - b)):
                w = int(slots[i, s]) & 0x1FFFFFFF
                assert w & 0xFFFFFF == g[colk][b + s]
                if key == "nbr":
                    q = int(g["ecode"][b + s])
                    assert w >> 24 == (q & 7) * 3 + (q >> 3)
