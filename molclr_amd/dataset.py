"""Synthetic molecular graphs and the MolCLR node-mask augmentation.

RDKit and the PubChem-10M SMILES file are not available here, so molecules
are generated directly in the reference's index space:

* atoms n ~ Uniform{10..50} ("uniform", configs c1-c4) or
  round(Normal(27, 9)) clipped to [6, 80] ("pubchem", config c5);
* topology: random recursive tree (atom i bonds to Uniform{0..i-1}) plus
  floor(n/8) ring-closure bonds between non-bonded pairs;
* atom type index = Z-1 (ATOM_LIST.index, dataset/dataset.py:26,75):
  C 0.72, N 0.12, O 0.11, F / S / Cl 0.015 each, Br 0.005;
* chirality {0: 0.96, 1: 0.02, 2: 0.02}; bond type {single .55, double .12,
  triple .01, aromatic .32}; bond dir {0: .98, 1: .01, 2: .01};
* every bond becomes the consecutive directed pair (s,e), (e,s) with the same
  [bond type, bond dir] (dataset/dataset.py:93-109).

Augmentation (dataset/dataset.py:111-145), independently per view: mask
max(1, floor(0.25 N)) atoms to [118, 0] (the mask token, len(ATOM_LIST)),
drop floor(0.25 M) bonds (both directions), keep the surviving edges in their
original order.  The reference uses Python's unseeded ``random``; here every
stream is a seeded numpy Generator so runs are reproducible.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

from .data import Batch, Data, collate_pairs
from .shards import read_smiles  # noqa: F401  (dataset/dataset.py:46-53)

MASK_ATOM = 118  # len(ATOM_LIST), dataset/dataset.py:123

_ATOM_IDX = np.array([5, 6, 7, 8, 15, 16, 34], dtype=np.int64)  # C N O F S Cl Br (Z-1)
_ATOM_P = np.array([0.72, 0.12, 0.11, 0.015, 0.015, 0.015, 0.005])
_CHIR_P = np.array([0.96, 0.02, 0.02])
_BT_P = np.array([0.55, 0.12, 0.01, 0.32])
_BD_P = np.array([0.98, 0.01, 0.01])


@dataclass
class Molecule:
    """Un-augmented molecule in the reference's tensor layout (numpy int64)."""
    x: np.ndarray           # [N, 2]
    edge_index: np.ndarray  # [2, 2M]
    edge_attr: np.ndarray   # [2M, 2]

    @property
    def num_atoms(self) -> int:
        return int(self.x.shape[0])

    @property
    def num_bonds(self) -> int:
        return int(self.edge_attr.shape[0] // 2)


def _num_atoms(rng: np.random.Generator, shape: str) -> int:
    if shape == "uniform":
        return int(rng.integers(10, 51))
    if shape == "pubchem":
        return int(min(80, max(6, round(rng.normal(27.0, 9.0)))))
    raise ValueError(f"unknown molecule size distribution {shape!r}")


def random_molecule(rng: np.random.Generator, shape: str = "uniform",
                    num_atoms: int | None = None) -> Molecule:
    n = _num_atoms(rng, shape) if num_atoms is None else int(num_atoms)
    bonds = []
    present = set()
    for i in range(1, n):
        j = int(rng.integers(0, i))
        bonds.append((j, i))
        present.add((j, i))
    extra = n // 8
    tries = 0
    while extra > 0 and tries < 100 * n:
        tries += 1
        a, b = (int(v) for v in rng.integers(0, n, size=2))
        if a == b:
            continue
        key = (min(a, b), max(a, b))
        if key in present:
            continue
        present.add(key)
        bonds.append(key)
        extra -= 1
    M = len(bonds)
    atom = _ATOM_IDX[rng.choice(len(_ATOM_IDX), size=n, p=_ATOM_P)]
    chir = rng.choice(3, size=n, p=_CHIR_P)
    x = np.stack([atom, chir], 1).astype(np.int64)
    bt = rng.choice(4, size=M, p=_BT_P)
    bd = rng.choice(3, size=M, p=_BD_P)
    b = np.asarray(bonds, dtype=np.int64).reshape(M, 2)
    row = np.empty(2 * M, dtype=np.int64)
    col = np.empty(2 * M, dtype=np.int64)
    row[0::2], col[0::2] = b[:, 0], b[:, 1]
    row[1::2], col[1::2] = b[:, 1], b[:, 0]
    attr = np.repeat(np.stack([bt, bd], 1).astype(np.int64), 2, axis=0)
    return Molecule(x, np.stack([row, col], 0), attr)


def mask_view(mol: Molecule, rng: np.random.Generator):
    """One augmented view, dataset/dataset.py:111-131 (returns numpy arrays)."""
    N, M = mol.num_atoms, mol.num_bonds
    num_mask_nodes = max(1, math.floor(0.25 * N))
    num_mask_edges = max(0, math.floor(0.25 * M))
    mask_nodes = rng.choice(N, size=num_mask_nodes, replace=False)
    mask_edges_single = rng.choice(M, size=num_mask_edges, replace=False) if M else np.zeros(0, int)
    x = mol.x.copy()
    x[mask_nodes] = (MASK_ATOM, 0)
    keep = np.ones(2 * M, dtype=bool)
    keep[2 * mask_edges_single] = False
    keep[2 * mask_edges_single + 1] = False
    return x, mol.edge_index[:, keep], mol.edge_attr[keep]


def augment_pair(mol: Molecule, rng_i: np.random.Generator, rng_j: np.random.Generator):
    """(Data_i, Data_j) as MoleculeDataset.__getitem__ returns (dataset.py:147)."""
    out = []
    for rng in (rng_i, rng_j):
        x, ei, ea = mask_view(mol, rng)
        out.append(Data(x=torch.from_numpy(x), edge_index=torch.from_numpy(ei),
                        edge_attr=torch.from_numpy(ea)))
    return tuple(out)


def collate_views(views) -> Batch:
    """Fast numpy collate of (x, edge_index, edge_attr) triples into a Batch
    (same result as Batch.from_data_list)."""
    sizes = np.array([v[0].shape[0] for v in views], dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(sizes)])
    x = np.concatenate([v[0] for v in views], 0)
    # C order, as PyG's collate yields it (a strided edge_index would cost
    # every consumer a copy)
    ei = np.ascontiguousarray(np.concatenate([v[1] + offs[g] for g, v in enumerate(views)], 1))
    ea = np.concatenate([v[2] for v in views], 0)
    batch = np.repeat(np.arange(len(views), dtype=np.int64), sizes)
    b = Batch(x=torch.from_numpy(x), edge_index=torch.from_numpy(ei),
              edge_attr=torch.from_numpy(ea), batch=torch.from_numpy(batch))
    b.ptr = torch.from_numpy(offs)
    b._num_graphs = len(views)
    return b


class SyntheticPairBatches:
    """Deterministic stream of (Batch_i, Batch_j) contrastive batches.

    Seeds: graph seed ``seed``, view seeds ``seed+1`` /
    ``seed+2``; give each data-parallel rank ``seed = rank * 10**6``.
    """

    def __init__(self, batch_size: int, seed: int = 0, shape: str = "uniform"):
        self.batch_size = batch_size
        self.shape = shape
        self.g = np.random.default_rng(seed)
        self.vi = np.random.default_rng(seed + 1)
        self.vj = np.random.default_rng(seed + 2)

    def molecules(self, n: int):
        return [random_molecule(self.g, self.shape) for _ in range(n)]

    def next(self):
        mols = self.molecules(self.batch_size)
        vi = [mask_view(m, self.vi) for m in mols]
        vj = [mask_view(m, self.vj) for m in mols]
        return collate_views(vi), collate_views(vj)

    def take(self, n: int):
        return [self.next() for _ in range(n)]


class MoleculeDataset(torch.utils.data.Dataset):
    """Map-style dataset of synthetic molecules with the reference's
    ``__getitem__ -> (Data_i, Data_j)`` contract (dataset/dataset.py:56-150).

    Views are drawn from ``SeedSequence([seed, rank, index, call])``: every
    (rank, molecule, epoch) pair gets its own augmentation stream."""

    def __init__(self, num_molecules: int, seed: int = 0, shape: str = "uniform", rank: int = 0):
        super().__init__()
        rng = np.random.default_rng(seed)
        self.mols = [random_molecule(rng, shape) for _ in range(num_molecules)]
        self.seed = seed
        self.rank = rank
        self._calls = 0

    def __getitem__(self, index):
        # per-item, per-call view streams: reproducible yet different each epoch
        self._calls += 1
        ss = np.random.SeedSequence([self.seed, self.rank, index, self._calls])
        ri, rj = (np.random.default_rng(s) for s in ss.spawn(2))
        return augment_pair(self.mols[index], ri, rj)

    def __len__(self):
        return len(self.mols)


class ShardedSubsetSampler(torch.utils.data.Sampler):
    """SubsetRandomSampler for data parallelism: every epoch, one permutation of
    ``indices`` seeded by (seed, epoch) -- the same on every rank -- is dealt
    round-robin, rank r taking positions r, r + world, ...; the tail that does
    not divide evenly is dropped, so every rank sees the same number of
    molecules (and of full batches, drop_last) and no molecule is seen by two
    ranks in one epoch.  world == 1 is SubsetRandomSampler with a seeded,
    per-epoch permutation (the reference's dataset/dataset.py:176-177)."""

    def __init__(self, indices, rank: int = 0, world: int = 1, seed: int = 0):
        if not 0 <= rank < world:
            raise ValueError(f"rank {rank} outside world size {world}")
        self.indices = list(indices)
        self.rank, self.world, self.seed = rank, world, seed
        self.epoch = 0

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def __iter__(self):
        per = len(self.indices) // self.world
        order = np.random.default_rng([self.seed, self.epoch]).permutation(len(self.indices))
        self.epoch += 1
        mine = order[self.rank:per * self.world:self.world]
        return iter([self.indices[i] for i in mine])

    def __len__(self):
        return len(self.indices) // self.world


def view_seed(seed: int, rank: int, epoch: int, batch: int) -> int:
    """The 64-bit key the device augmentation draws a batch's subsets from:
    distinct for every (seed, rank, epoch, batch), so a molecule gets new
    views every epoch and the same ones on a rerun."""
    z = 0
    for v in (seed, rank, epoch, batch):
        z = (z ^ (int(v) & _M64)) * 0x9E3779B97F4A7C15 & _M64
        z ^= z >> 29
    return z


_M64 = (1 << 64) - 1
AUG_MODES = ("node", "subgraph", "mix")


class DeviceViewLoader:
    """The DataLoader of the device path: every batch is ``batch_size``
    molecule ids from ``sampler`` (drop_last, dataset/dataset.py:179-183) and
    both views are built on the GPU from the resident
    :class:`~molclr_amd.augment.DeviceMoleculeStore` -- node masking
    (dataset.py:111-147), subgraph removal (dataset_subgraph.py:96-177) or
    both (dataset_mix.py:86-217), collated into the Batch fields.  Yields the
    (Batch_i, Batch_j) pairs ``MolCLR.train`` iterates over
    (molclr.py:108), already on the device."""

    def __init__(self, store, sampler, batch_size: int, aug: str = "node", seed: int = 0,
                 rank: int = 0):
        if aug not in AUG_MODES:
            raise ValueError(f"aug {aug!r}: one of {AUG_MODES}")
        self.store, self.sampler = store, sampler
        self.batch_size, self.aug, self.seed, self.rank = int(batch_size), aug, seed, rank
        self.epoch = 0
        # optional callback(sizes, graphs_i, graphs_j) called when an epoch's
        # batches are drawn, before the first is built, with the (nodes, edges)
        # of every batch pair of the epoch (node masking: exact; subgraph / mix:
        # exact nodes, the un-dropped bond count as the edge bound);
        # MolCLR.train hands it to the HIP-graph step
        self.on_epoch_plan = None

    def __len__(self):
        return len(self.sampler) // self.batch_size

    def __iter__(self):
        ids = np.fromiter(iter(self.sampler), dtype=np.int64)
        epoch = self.epoch
        self.epoch += 1
        bs = self.batch_size
        nb = ids.shape[0] // bs
        if self.on_epoch_plan is not None and nb:
            sizes = []
            for b in range(nb):
                sel = ids[b * bs:(b + 1) * bs]
                if self.aug == "node":
                    n, e = self.store.mask_view_size(sel)
                else:  # subgraph / mix keep every atom and drop bonds: e is a bound
                    n, e = int(self.store.num_atoms[sel].sum()), 2 * int(self.store.num_bonds[sel].sum())
                sizes.append((2 * n, 2 * e))
            self.on_epoch_plan(sizes, bs, bs)
        for b in range(nb):
            host = ids[b * bs:(b + 1) * bs]
            key = view_seed(self.seed, self.rank, epoch, b)
            self.last = (host, key)   # the batch's molecule ids and subset key
            if self.aug == "node":
                yield self.store.mask_views(host, key, host_ids=host)
            else:
                yield self.store.aug_views(host, key, mode=self.aug, host_ids=host)


class MoleculeDatasetWrapper:
    """dataset/dataset.py:153-185 (and the subgraph / mix modules' copies):
    a shuffled train / valid split and loaders of full batches (drop_last:
    NT-Xent needs them).

    ``data_path`` is what config.yaml names (config.yaml:27):

    * a SMILES text file, read as ``read_smiles`` does (dataset.py:46-53: the
      last comma-separated field of every line), featurised once into a
      cached binary shard next to it (molclr_amd.shards; with explicit
      hydrogens for ``aug: mix``, whose module calls ``Chem.AddHs``,
      dataset_mix.py:87-88);
    * a binary graph shard (molclr_amd.shards);
    * ``synthetic:<num_molecules>`` (SURVEY §8d generator).

    ``aug`` picks the augmentation (molclr.py:184-191).  ``views='device'``
    (default) keeps the molecules resident in HBM and builds both views of
    every batch on the GPU (:class:`DeviceViewLoader`); ``views='host'`` is
    the reference's DataLoader of host-built node-mask views
    (``aug: node`` only).

    Data parallel: with ``torch.distributed`` initialised (or ``rank`` /
    ``world`` given), each rank draws a disjoint, equally sized shard of the
    train and valid index sets every epoch (ShardedSubsetSampler)."""

    def __init__(self, batch_size, num_workers, valid_size, data_path, seed: int = 0,
                 shape: str = "uniform", rank: int | None = None, world: int | None = None,
                 aug: str = "node", views: str = "device"):
        if aug not in AUG_MODES:
            raise ValueError("Not defined molecule augmentation!")
        if views not in ("device", "host"):
            raise ValueError(f"views {views!r}: 'device' or 'host'")
        if views == "host" and aug != "node":
            raise ValueError(f"aug {aug!r} views are built on the device only (views='device')")
        self.batch_size = batch_size
        self.num_workers = num_workers
        self.valid_size = valid_size
        self.data_path = data_path
        self.seed = seed
        self.shape = shape
        self.rank, self.world = rank, world
        self.aug, self.views = aug, views

    def _rank_world(self) -> tuple[int, int]:
        if self.rank is not None and self.world is not None:
            return int(self.rank), int(self.world)
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank(), dist.get_world_size()
        return 0, 1

    def _num_molecules(self) -> int:
        return int(str(self.data_path).split(":", 1)[1])

    def shard_path(self):
        """The binary shard behind ``data_path`` (featurising a SMILES file
        once), or None for synthetic data."""
        from .shards import cached_smiles_shard, is_shard
        p = str(self.data_path)
        if p.startswith("synthetic:"):
            return None
        if is_shard(p):
            return p
        return cached_smiles_shard(p, add_hs=(self.aug == "mix"))

    def get_data_loaders(self):
        rank, _ = self._rank_world()
        shard = self.shard_path()
        if self.views == "device":
            store = self.device_store(shard)
            return self.get_train_validation_data_loaders(store, len_=store.num_molecules)
        if shard is None:
            train_dataset = MoleculeDataset(self._num_molecules(), self.seed, self.shape, rank=rank)
        else:
            from .shards import ShardMoleculeDataset
            train_dataset = ShardMoleculeDataset(shard, seed=self.seed, rank=rank)
        return self.get_train_validation_data_loaders(train_dataset)

    def device_store(self, shard=None):
        """The whole dataset resident on the current GPU (every rank holds it:
        10 M PubChem molecules take ~28 GB of the 288 GB)."""
        from .augment import DeviceMoleculeStore
        if not torch.cuda.is_available():
            raise RuntimeError("device views need a GPU (views='host' for the CPU DataLoader)")
        dev = torch.device("cuda", torch.cuda.current_device())
        if shard is None:
            rng = np.random.default_rng(self.seed)
            mols = [random_molecule(rng, self.shape) for _ in range(self._num_molecules())]
            return DeviceMoleculeStore.from_molecules(mols, dev)
        from .shards import GraphShard
        return GraphShard(shard).device_store(dev)

    def get_train_validation_data_loaders(self, train_dataset, len_: int | None = None):
        rank, world = self._rank_world()
        num_train = len(train_dataset) if len_ is None else len_
        indices = np.random.default_rng(self.seed).permutation(num_train).tolist()
        # every molecule takes part in every aug mode, as in the reference
        # (large ones run the subgraph / mix plan from a global workspace)
        split = int(np.floor(self.valid_size * num_train))
        train_idx, valid_idx = indices[split:], indices[:split]
        train_sampler = ShardedSubsetSampler(train_idx, rank, world, seed=self.seed + 1)
        valid_sampler = ShardedSubsetSampler(valid_idx, rank, world, seed=self.seed + 2)
        if self.views == "device":
            return (DeviceViewLoader(train_dataset, train_sampler, self.batch_size, self.aug,
                                     self.seed + 1, rank),
                    DeviceViewLoader(train_dataset, valid_sampler, self.batch_size, self.aug,
                                     self.seed + 2, rank))
        kw = dict(batch_size=self.batch_size, num_workers=self.num_workers, drop_last=True,
                  collate_fn=collate_pairs)
        train_loader = torch.utils.data.DataLoader(train_dataset, sampler=train_sampler, **kw)
        valid_loader = torch.utils.data.DataLoader(train_dataset, sampler=valid_sampler, **kw)
        return train_loader, valid_loader
