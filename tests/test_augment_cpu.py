"""Oracle of the on-device node-mask augmentation + collate (oracle/augment_ref.py):
the vectorised form against the reference's own per-molecule loop
(dataset/dataset.py:111-131) and PyG collate, subset sizes and uniformity."""
import numpy as np
import torch

from molclr_amd.data import Batch, Data
from molclr_amd.dataset import random_molecule
from oracle.augment_ref import (MASK_ATOM, chosen_items, mask_views, num_masked,
                                reference_mask_view)


def _store(mols):
    xs = [m.x for m in mols]
    eis = [m.edge_index for m in mols]
    eas = [m.edge_attr for m in mols]
    return {
        "x": np.concatenate(xs, 0),
        "atom_ptr": np.concatenate([[0], np.cumsum([x.shape[0] for x in xs])]),
        "edge_index": np.concatenate(eis, 1),
        "edge_attr": np.concatenate(eas, 0),
        "bond_ptr": np.concatenate([[0], np.cumsum([e.shape[1] // 2 for e in eis])]),
    }


def test_subset_sizes_follow_the_reference():
    # dataset.py:111-112
    assert num_masked(1, 0) == (1, 0)
    assert num_masked(7, 3) == (1, 0)
    assert num_masked(8, 4) == (2, 1)
    assert num_masked(50, 55) == (12, 13)
    for n in range(1, 40):
        for k in (0, 1, n // 4, n):
            s = chosen_items(5, 0, 0, 17, n, k)
            assert len(s) == min(k, n) and len(set(s.tolist())) == len(s)
            assert np.all(np.diff(s) > 0) and (len(s) == 0 or (s[0] >= 0 and s[-1] < n))


def test_subsets_are_uniform_and_independent_per_view():
    n, k, trials = 10, 2, 4000
    freq = np.zeros(n)
    same = 0
    for seed in range(trials):
        a = chosen_items(seed, 0, 0, 3, n, k)
        b = chosen_items(seed, 1, 0, 3, n, k)
        freq[a] += 1
        same += int(np.array_equal(a, b))
    p = k / n
    sigma = np.sqrt(trials * p * (1 - p))
    assert np.all(np.abs(freq - trials * p) < 5 * sigma), freq
    # P(two independent 2-subsets of 10 agree) = 1/45
    assert abs(same - trials / 45) < 5 * np.sqrt(trials / 45)


def test_vectorised_oracle_matches_reference_loop_and_collate():
    rng = np.random.default_rng(3)
    mols = [random_molecule(rng) for _ in range(12)]
    store = _store(mols)
    ids = np.array([4, 0, 11, 4, 7], dtype=np.int64)  # repeats allowed (sampling with replacement)
    for view in (0, 1):
        out = mask_views(store, ids, seed=123, view=view)
        datas = []
        for mid, (mn, me) in zip(ids, out["masks"]):
            m = mols[mid]
            assert (len(mn), len(me)) == num_masked(m.num_atoms, m.num_bonds)
            x, ei, ea = reference_mask_view(m.x.tolist(), m.edge_index.tolist(),
                                            m.edge_attr.tolist(), mn.tolist(), me.tolist())
            datas.append(Data(x=torch.tensor(x), edge_index=torch.tensor(ei).view(2, -1),
                              edge_attr=torch.tensor(ea).view(-1, 2)))
        ref = Batch.from_data_list(datas)
        assert np.array_equal(out["x"], ref.x.numpy())
        assert np.array_equal(out["edge_index"], ref.edge_index.numpy())
        assert np.array_equal(out["edge_attr"], ref.edge_attr.numpy())
        assert np.array_equal(out["batch"], ref.batch.numpy())
        assert np.array_equal(out["ptr"], ref.ptr.numpy())
        assert (out["x"][:, 0] == MASK_ATOM).sum() >= len(ids)


def test_edge_cases():
    # one atom / no bonds; one bond (floor(1/4) = 0 dropped); three bonds
    class M:
        def __init__(self, n, bonds):
            self.x = np.stack([np.arange(n) % 5, np.zeros(n, np.int64)], 1).astype(np.int64)
            ei = []
            for s, e in bonds:
                ei += [(s, e), (e, s)]
            self.edge_index = np.array(ei, dtype=np.int64).reshape(-1, 2).T.copy()
            self.edge_attr = np.repeat(np.arange(len(bonds)) % 4, 2)[:, None].repeat(2, 1)
    mols = [M(1, []), M(2, [(0, 1)]), M(4, [(0, 1), (1, 2), (2, 3)])]
    store = _store(mols)
    out = mask_views(store, np.array([0, 1, 2]), seed=0, view=0)
    assert out["x"].shape == (7, 2) and out["edge_index"].shape == (2, 2 + 6)
    assert np.array_equal(out["x"][0], [MASK_ATOM, 0])  # the only atom is always masked
    assert np.array_equal(out["ptr"], [0, 1, 3, 7])
    empty = mask_views(store, np.zeros(0, np.int64), seed=0, view=0)
    assert empty["x"].shape == (0, 2) and np.array_equal(empty["ptr"], [0])


def test_streams_do_not_alias_across_seed_view_kind():
    """A flat seed ^ (2 view + kind) key made view 1 at seed s replay view 0 at
    seed s ^ 2 (and the bond stream of one view replay the atom stream of the
    next seed); the chained splitmix64 keys of augment.hip do not."""
    from oracle.augment_ref import _stream
    keys = {}
    for seed in range(64):
        for view in (0, 1):
            for kind in (0, 1):
                k = int(_stream(seed, view, kind, 7))
                assert k not in keys, (seed, view, kind, keys.get(k))
                keys[k] = (seed, view, kind)
    n, k = 40, 10
    for s in range(32):
        assert not np.array_equal(chosen_items(s, 1, 0, 3, n, k), chosen_items(s ^ 2, 0, 0, 3, n, k))
