"""ORACLE — test infrastructure only (see oracle/__init__.py).

CPU restatement of the on-device augmentation + collate of
molclr_amd/csrc/augment.hip: the node-mask views (``molclr_mask_views``,
below) and, at the end of the file, the subgraph-removal and mixed views
(``molclr_aug_views_*``, dataset_subgraph.py / dataset_mix.py).  Node mask, in
two layers:

* :func:`reference_mask_view` follows the reference's per-molecule loop in
  MoleculeDataset.__getitem__ literally (dataset/dataset.py:111-131): given the
  masked atom and bond index lists it sets ``x[atom] = [len(ATOM_LIST), 0]``
  and copies every directed edge ``bond_idx`` of ``range(2M)`` not in
  ``[2i for i in mask] + [2i+1 for i in mask]``, in order.  Pure Python loops:
  small cases only.
* :func:`mask_views` is the vectorised numpy form used against the kernel at
  batch size: the same subset keys as the kernel (splitmix64 of seed, view,
  molecule id, item; the k smallest keys, ties by index), then the masking
  above, then PyG 1.6.3's ``Batch.from_data_list`` collate (x / edge_attr
  concatenated, edge_index offset by the running atom count, ascending
  ``batch``, ``ptr``).

The reference draws its subsets with Python's unseeded ``random.sample``
(dataset.py:113-116), so no reference stream exists to match: the subset
RNG is "parity unpinned" by construction, and the tests check what the
reference specifies -- subset sizes max(1, floor(0.25 N)) / floor(0.25 M),
uniformity, and the masking/collate given the subsets (bit-exact).
"""
from __future__ import annotations

import numpy as np

MASK_ATOM = 118  # len(ATOM_LIST), dataset/dataset.py:123
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def _stream(seed: int, view: int, kind: int, mol_id: int) -> np.uint64:
    """augment.hip subset_stream: splitmix64 chained over (seed, view, kind, id)."""
    z = splitmix64(np.uint64(seed))
    z = splitmix64(z ^ np.uint64(view))
    z = splitmix64(z ^ np.uint64(kind))
    return splitmix64(z ^ np.uint64(mol_id))


def chosen_items(seed: int, view: int, kind: int, mol_id: int, n: int, k: int) -> np.ndarray:
    """Indices (ascending) of the k smallest keys among n items, ties by index."""
    if k <= 0 or n <= 0:
        return np.zeros(0, dtype=np.int64)
    if k >= n:
        return np.arange(n, dtype=np.int64)
    keys = splitmix64(_stream(seed, view, kind, mol_id) ^ np.arange(n, dtype=np.uint64))
    order = np.lexsort((np.arange(n), keys))  # by key, then index
    return np.sort(order[:k]).astype(np.int64)


def num_masked(n_atoms: int, n_bonds: int) -> tuple[int, int]:
    """dataset.py:111-112: max(1, floor(0.25 N)) atoms, max(0, floor(0.25 M)) bonds."""
    return (max(1, n_atoms // 4) if n_atoms > 0 else 0), n_bonds // 4


def reference_mask_view(x, edge_index, edge_attr, mask_nodes, mask_edges_single):
    """dataset/dataset.py:117-131, loop for loop (lists of ints in, lists out)."""
    M = len(edge_attr) // 2
    mask_edges = [2 * i for i in mask_edges_single] + [2 * i + 1 for i in mask_edges_single]
    x_i = [list(r) for r in x]
    for atom_idx in mask_nodes:
        x_i[atom_idx] = [MASK_ATOM, 0]
    ei = [[], []]
    ea = []
    for bond_idx in range(2 * M):
        if bond_idx not in mask_edges:
            ei[0].append(edge_index[0][bond_idx])
            ei[1].append(edge_index[1][bond_idx])
            ea.append(list(edge_attr[bond_idx]))
    return x_i, ei, ea


def mask_views(store: dict, mol_ids, seed: int, view: int) -> dict:
    """Batch fields of one view: x [N,2], edge_index [2,E], edge_attr [E,2],
    batch [N], ptr [B+1] (int64), plus the chosen subsets per molecule."""
    sx = np.asarray(store["x"], dtype=np.int64)
    aptr = np.asarray(store["atom_ptr"], dtype=np.int64)
    sei = np.asarray(store["edge_index"], dtype=np.int64)
    sea = np.asarray(store["edge_attr"], dtype=np.int64)
    bptr = np.asarray(store["bond_ptr"], dtype=np.int64)
    xs, eis, eas, bs, ptr = [], [], [], [], [0]
    masks = []
    for g, mid in enumerate(np.asarray(mol_ids, dtype=np.int64)):
        a0, a1 = aptr[mid], aptr[mid + 1]
        b0, b1 = bptr[mid], bptr[mid + 1]
        n, M = int(a1 - a0), int(b1 - b0)
        ka, kb = num_masked(n, M)
        mn = chosen_items(seed, view, 0, int(mid), n, ka)
        me = chosen_items(seed, view, 1, int(mid), M, kb)
        x = sx[a0:a1].copy()
        x[mn] = (MASK_ATOM, 0)
        keep = np.ones(2 * M, dtype=bool)
        keep[2 * me] = False
        keep[2 * me + 1] = False
        ei = sei[:, 2 * b0:2 * b1][:, keep] + ptr[-1]
        xs.append(x)
        eis.append(ei)
        eas.append(sea[2 * b0:2 * b1][keep])
        bs.append(np.full(n, g, dtype=np.int64))
        ptr.append(ptr[-1] + n)
        masks.append((mn, me))
    return {
        "x": np.concatenate(xs, 0) if xs else np.zeros((0, 2), np.int64),
        "edge_index": np.concatenate(eis, 1) if eis else np.zeros((2, 0), np.int64),
        "edge_attr": np.concatenate(eas, 0) if eas else np.zeros((0, 2), np.int64),
        "batch": np.concatenate(bs) if bs else np.zeros(0, np.int64),
        "ptr": np.asarray(ptr, dtype=np.int64),
        "masks": masks,
    }


# ---------------------------------------------------------------------------
# Subgraph removal (dataset/dataset_subgraph.py:70-177) and the mixed views
# (dataset/dataset_mix.py:46-217), restated with plain ordered dicts in place
# of networkx (nx.Graph(edges): nodes in order of first appearance, each
# node's neighbours in insertion order; remove_node drops a node from its
# neighbours' dicts) and Python's own set for the frontier.
# ---------------------------------------------------------------------------
AUG_SUBGRAPH, AUG_MIX = 0, 1


def bond_graph(bonds):
    """nx.Graph(edges) as {node: {neighbour: None}} in networkx's orders."""
    adj = {}
    for s, e in bonds:
        adj.setdefault(s, {})
        adj.setdefault(e, {})
        adj[s][e] = None
        adj[e][s] = None
    return adj


def graph_copy(adj):
    """Graph.copy() (dataset_subgraph.py:72 / dataset_mix.py:48): networkx
    re-adds every edge (u, v) walking u in node order and v in u's order, so
    a node's neighbours become those earlier in node order (in node order),
    then the later ones in their original order."""
    G = {u: {} for u in adj}
    for u, nbrs in adj.items():
        for v in nbrs:
            G[u].setdefault(v, None)
            G[v].setdefault(u, None)
    return G


def remove_subgraph(adj, center, percent, guard=True):
    """removeSubgraph (dataset_subgraph.py:70-88) / remove_subgraph
    (dataset_mix.py:46-68, with the empty-frontier guard at :55-56).  Returns
    (remaining graph, removed list, guard_hit).  A centre outside the bond
    graph is taken as a frontier of one isolated atom (the reference raises)."""
    G = graph_copy(adj)
    num = int(np.floor(len(G) * percent))
    removed, temp, hit = [], [center], False
    while len(removed) < num:
        if len(temp) < 1:
            hit = True
            if guard:
                break
            raise RuntimeError("removeSubgraph would not terminate")
        neighbors = []
        for n in temp:
            neighbors.extend([i for i in G.get(n, {}) if i not in temp])
        for n in temp:
            if len(removed) < num:
                for v in G.pop(n, {}):
                    G[v].pop(n, None)
                removed.append(n)
            else:
                break
        temp = list(set(neighbors))
    return G, removed, hit


def graph_edges(G):
    """list(G.edges) of an undirected networkx graph: each edge once, from the
    endpoint that comes first in node order."""
    seen, out = set(), []
    for u, nbrs in G.items():
        for v in nbrs:
            if v not in seen:
                out.append((u, v))
        seen.add(u)
    return out


def _u53(z) -> float:
    return float(int(z) >> 11) * 2.0 ** -53


def aug_centres(seed: int, mol_id: int, n: int) -> tuple[int, int]:
    """random.sample(range(N), 2) as augment.hip draws it: the atoms with the
    smallest and second smallest key of the molecule's centre stream."""
    if n < 2:
        return 0, 0
    keys = splitmix64(_stream(seed, 2, 2, mol_id) ^ np.arange(n, dtype=np.uint64))
    order = np.lexsort((np.arange(n), keys))
    return int(order[0]), int(order[1])


def aug_percent(seed: int, view: int, mol_id: int, mode: int) -> float:
    """0.25 (subgraph) or random.uniform(0, 0.2) (mix) from a per-view key."""
    if mode == AUG_SUBGRAPH:
        return 0.25
    return 0.2 * _u53(splitmix64(_stream(seed, view, 3, mol_id)))


def aug_molecule(x, edge_index, edge_attr, seed, view, mol_id, mode):
    """One molecule's view: (x [N,2], kept directed-edge mask [2M], flags)."""
    n = x.shape[0]
    M = edge_index.shape[1] // 2
    bonds = [(int(edge_index[0, 2 * b]), int(edge_index[1, 2 * b])) for b in range(M)]
    adj = bond_graph(bonds)
    c = aug_centres(seed, mol_id, n)[view]
    pct = aug_percent(seed, view, mol_id, mode)
    G, removed, hit = remove_subgraph(adj, c, pct, guard=True)
    edges = graph_edges(G)
    eset = set(edges)
    if mode == AUG_SUBGRAPH:   # dataset_subgraph.py:150-160: (start, end) only
        keep_b = [(s, e) in eset for s, e in bonds]
    else:                      # dataset_mix.py:157-167: either orientation
        keep_b = [(s, e) in eset or (e, s) in eset for s, e in bonds]
    x = x.copy()
    rem = set(removed)
    masked = set(removed)
    if mode == AUG_MIX:        # dataset_mix.py:174-189
        remain = [i for i in range(n) if i not in rem]
        ka = max(0, n // 4 - len(removed))
        for p in chosen_items(seed, view, 4, mol_id, len(remain), ka):
            masked.add(remain[p])
        kept = [b for b in range(M) if keep_b[b]]
        kb = max(0, len(kept) - (3 * M + 3) // 4)
        for p in chosen_items(seed, view, 5, mol_id, len(kept), kb):
            keep_b[kept[p]] = False
    for i in masked:
        x[i] = (MASK_ATOM, 0)
    keep = np.repeat(np.asarray(keep_b, dtype=bool), 2)
    center_in = c in adj or int(np.floor(len(adj) * pct)) == 0
    return x, keep, {"guard": hit, "centre_outside": not center_in, "removed": removed}


def aug_views(store: dict, mol_ids, seed: int, view: int, mode: int) -> dict:
    """Batch fields of one subgraph / mix view (molclr_aug_views_*)."""
    sx = np.asarray(store["x"], dtype=np.int64)
    aptr = np.asarray(store["atom_ptr"], dtype=np.int64)
    sei = np.asarray(store["edge_index"], dtype=np.int64)
    sea = np.asarray(store["edge_attr"], dtype=np.int64)
    bptr = np.asarray(store["bond_ptr"], dtype=np.int64)
    xs, eis, eas, bs, ptr, flags = [], [], [], [], [0], []
    for g, mid in enumerate(np.asarray(mol_ids, dtype=np.int64)):
        a0, a1 = aptr[mid], aptr[mid + 1]
        b0, b1 = bptr[mid], bptr[mid + 1]
        x, keep, fl = aug_molecule(sx[a0:a1], sei[:, 2 * b0:2 * b1], sea[2 * b0:2 * b1], seed,
                                   view, int(mid), mode)
        xs.append(x)
        eis.append(sei[:, 2 * b0:2 * b1][:, keep] + ptr[-1])
        eas.append(sea[2 * b0:2 * b1][keep])
        bs.append(np.full(a1 - a0, g, dtype=np.int64))
        ptr.append(ptr[-1] + int(a1 - a0))
        flags.append(fl)
    return {
        "x": np.concatenate(xs, 0) if xs else np.zeros((0, 2), np.int64),
        "edge_index": np.concatenate(eis, 1) if eis else np.zeros((2, 0), np.int64),
        "edge_attr": np.concatenate(eas, 0) if eas else np.zeros((0, 2), np.int64),
        "batch": np.concatenate(bs) if bs else np.zeros(0, np.int64),
        "ptr": np.asarray(ptr, dtype=np.int64),
        "flags": flags,
    }
