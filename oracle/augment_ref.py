"""ORACLE — test infrastructure only (see oracle/__init__.py).

CPU restatement of the on-device node-mask augmentation + collate
(``molclr_mask_views``, molclr_amd/csrc/augment.hip), in two layers:

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
