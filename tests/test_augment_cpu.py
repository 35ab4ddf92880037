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


# ---------------------------------------------------------------------------
# Subgraph-removal / mixed views (dataset_subgraph.py, dataset_mix.py)
# ---------------------------------------------------------------------------
def _pyset_emulated(items):
    """The CPython set-of-small-ints model augment.hip's pyset_order
    implements (open addressing, 10-slot linear probes while i + 9 <= mask,
    perturbation i = 5 i + 1 + (perturb >>= 5), growth to the next power of
    two above 4 x used when fill x 5 >= mask x 3, old-slot-order reinsertion)."""
    mask, table, fill = 7, [None] * 8, 0

    def insert_clean(k):
        i, perturb = k & mask, k
        while True:
            if table[i] is None:
                table[i] = k
                return
            if i + 9 <= mask:
                for j in range(i + 1, i + 10):
                    if table[j] is None:
                        table[j] = k
                        return
            perturb >>= 5
            i = (i * 5 + 1 + perturb) & mask

    for k in items:
        i, perturb, inserted = k & mask, k, False
        while True:
            last = i + 9 if i + 9 <= mask else i
            done = False
            for j in range(i, last + 1):
                if table[j] is None:
                    table[j], inserted, done = k, True, True
                    break
                if table[j] == k:
                    done = True
                    break
            if done:
                break
            perturb >>= 5
            i = (i * 5 + 1 + perturb) & mask
        if inserted:
            fill += 1
            if fill * 5 >= mask * 3:
                old = [v for v in table if v is not None]
                size = 8
                while size <= fill * 4:
                    size <<= 1
                mask, table = size - 1, [None] * size
                for v in old:
                    insert_clean(v)
    return [v for v in table if v is not None]


def test_cpython_set_order_model():
    """The frontier order the kernel emulates is CPython's own list(set(x))."""
    rng = np.random.default_rng(0)
    for _ in range(3000):
        n = int(rng.integers(0, 160))
        hi = int(rng.choice([8, 40, 256]))
        items = [int(v) for v in rng.integers(0, hi, size=n)]
        assert _pyset_emulated(items) == list(set(items)), items


def _nx_remove_subgraph(edges, center, percent):
    """The reference loop run on networkx itself (guarded like
    dataset_mix.py:55-56)."""
    import networkx as nx
    G = nx.Graph(edges).copy()
    num = int(np.floor(len(G.nodes) * percent))
    removed, temp = [], [center]
    while len(removed) < num:
        if len(temp) < 1:
            break
        neighbors = []
        for n in temp:
            neighbors.extend([i for i in G.neighbors(n) if i not in temp])
        for n in temp:
            if len(removed) < num:
                G.remove_node(n)
                removed.append(n)
            else:
                break
        temp = list(set(neighbors))
    return G, removed


def test_subgraph_oracle_matches_networkx():
    """oracle/augment_ref.py's dict restatement of nx.Graph / neighbours /
    remove_node / G.edges against networkx 3 on random molecule graphs."""
    from oracle.augment_ref import bond_graph, graph_edges, remove_subgraph
    rng = np.random.default_rng(1)
    for t in range(300):
        m = random_molecule(rng, "pubchem" if t % 2 else "uniform")
        M = m.edge_attr.shape[0] // 2
        bonds = [(int(m.edge_index[0, 2 * b]), int(m.edge_index[1, 2 * b])) for b in range(M)]
        if t % 3 == 0:  # reversed orientations: networkx reports edges from the earlier node
            bonds = [(e, s) if (s + e + t) % 2 else (s, e) for s, e in bonds]
        pct = float(rng.choice([0.25, 0.2 * rng.random(), 0.9]))
        center = int(rng.integers(0, m.x.shape[0]))
        G_nx, rem_nx = _nx_remove_subgraph(bonds, center, pct)
        G_o, rem_o, _ = remove_subgraph(bond_graph(bonds), center, pct)
        assert rem_o == rem_nx
        assert graph_edges(G_o) == list(G_nx.edges)


def test_aug_views_oracle_properties():
    """Sizes and invariants of the subgraph / mix views (the reference's
    counts: floor(p x atoms-in-bonds) removed; mix tops masks up to floor(N/4)
    atoms and keeps at most ceil(3M/4) bonds)."""
    from oracle.augment_ref import AUG_MIX, AUG_SUBGRAPH, aug_centres, aug_views
    rng = np.random.default_rng(2)
    mols = [random_molecule(rng, "uniform") for _ in range(64)]
    st = _store(mols)
    ids = np.arange(64)
    for mode in (AUG_SUBGRAPH, AUG_MIX):
        v0, v1 = aug_views(st, ids, 5, 0, mode), aug_views(st, ids, 5, 1, mode)
        for v in (v0, v1):
            for g, m in enumerate(mols):
                n, M = m.x.shape[0], m.edge_attr.shape[0] // 2
                a0, a1 = v["ptr"][g], v["ptr"][g + 1]
                masked = int((v["x"][a0:a1, 0] == MASK_ATOM).sum())
                rem = v["flags"][g]["removed"]
                if mode == AUG_SUBGRAPH:
                    assert len(rem) == int(np.floor(n * 0.25))  # connected: all atoms in bonds
                    assert masked == len(rem)
                else:
                    assert masked == max(n // 4, len(rem))
                    kept = int((v["batch"][v["edge_index"][0]] == g).sum()) // 2
                    assert kept <= max((3 * M + 3) // 4, 0) or kept == 0
                assert not v["flags"][g]["guard"]
        for g, m in enumerate(mols):
            c0, c1 = aug_centres(5, g, m.x.shape[0])
            assert c0 != c1
