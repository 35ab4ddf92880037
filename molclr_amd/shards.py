"""Binary graph shards: the on-disk molecule format.

The reference reads ``pubchem-10m-clean.txt`` (config.yaml:27) one SMILES per
line (``read_smiles``, dataset/dataset.py:46-53) and featurises every molecule
with RDKit inside ``__getitem__`` on every access (dataset.py:61-109), 12
worker processes per GPU.  Here featurisation happens once (``featurise``,
molclr_amd/smiles.py, or the synthetic generator) and the result is stored as
a pre-featurised, memory-mappable shard that loads straight into a
:class:`~molclr_amd.augment.DeviceMoleculeStore` -- no per-step host work.

Layout (little endian, every array 64-byte aligned)::

    magic  b"MOLCLRG1"          8 bytes
    header u32 version (1), u32 flags (bit 0: hydrogens explicit, Chem.AddHs),
           u64 num_mols, u64 num_atoms, u64 num_bonds
    atom_ptr  i64 [num_mols + 1]     atoms of molecule g: [atom_ptr[g], atom_ptr[g+1])
    bond_ptr  i64 [num_mols + 1]     bonds of molecule g
    atoms     u8  [num_atoms, 2]     (atom type = ATOM_LIST index, chirality index)
    bonds     u16 [num_bonds, 2]     molecule-local (begin, end) atom of every bond
    battr     u8  [num_bonds, 2]     (BOND_LIST index, BONDDIR_LIST index)

which is the reference's featurisation (dataset.py:74-109) with every bond
kept once: the directed pair (begin, end), (end, begin) with the same
attributes is expanded when the shard is read, in the reference's order.
At PubChem scale (10 M molecules of ~27 atoms / ~29 bonds) a shard is ~1.5 GB;
the device store built from it (int64, the kernels' layout) ~28 GB, a tenth of
one MI355X's HBM.
"""
from __future__ import annotations

import os
import struct
from pathlib import Path
from typing import Iterable, Sequence

import numpy as np
import torch

MAGIC = b"MOLCLRG1"
VERSION = 1
_HDR = struct.Struct("<8sIIQQQ")
_ALIGN = 64

FLAG_EXPLICIT_H = 1   # molecules featurised after Chem.AddHs (dataset_mix.py:87-88)

MAX_ATOM_TYPE = 119   # 118 elements + the mask token (ginet_molclr.py:9)
MAX_CHIRALITY = 4     # CHIRALITY_LIST (dataset.py:27-32)
MAX_BOND_TYPE = 4     # BOND_LIST (dataset.py:33)
MAX_BOND_DIR = 3      # BONDDIR_LIST (dataset.py:34-38)


def _pad(n: int) -> int:
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


def _layout(num_mols: int, num_atoms: int, num_bonds: int) -> dict:
    off = _pad(_HDR.size)
    lay = {}
    for name, nbytes in (("atom_ptr", 8 * (num_mols + 1)), ("bond_ptr", 8 * (num_mols + 1)),
                         ("atoms", 2 * num_atoms), ("bonds", 4 * num_bonds),
                         ("battr", 2 * num_bonds)):
        lay[name] = off
        off = _pad(off + nbytes)
    lay["end"] = off
    return lay


def write_shard(path, molecules: Iterable, flags: int = 0) -> int:
    """Write molecules (objects with ``x`` [N,2], ``edge_index`` [2,2M] local,
    ``edge_attr`` [2M,2] holding every bond as the consecutive directed pair
    (s,e),(e,s), e.g. dataset.Molecule) as one shard; returns the count.
    ``flags``: FLAG_EXPLICIT_H when the molecules carry their hydrogens."""
    mols = list(molecules)
    xs, bonds, battr = [], [], []
    for m in mols:
        x = np.asarray(m.x, dtype=np.int64).reshape(-1, 2)
        ei = np.asarray(m.edge_index, dtype=np.int64).reshape(2, -1)
        ea = np.asarray(m.edge_attr, dtype=np.int64).reshape(-1, 2)
        if ei.shape[1] % 2 or ea.shape[0] != ei.shape[1]:
            raise ValueError("edge_index / edge_attr must hold directed pairs")
        fwd, rev = ei[:, 0::2], ei[:, 1::2]
        if not (np.array_equal(fwd[0], rev[1]) and np.array_equal(fwd[1], rev[0])
                and np.array_equal(ea[0::2], ea[1::2])):
            raise ValueError("every bond must be the pair (s,e),(e,s) with equal attributes "
                             "(dataset/dataset.py:93-109)")
        n = x.shape[0]
        if n > 0xFFFF or (fwd.size and (fwd.min() < 0 or fwd.max() >= n)):
            raise ValueError("atom index out of range for a u16 molecule-local index")
        if x.size and (x[:, 0].min() < 0 or x[:, 0].max() >= MAX_ATOM_TYPE
                       or x[:, 1].min() < 0 or x[:, 1].max() >= MAX_CHIRALITY):
            raise ValueError("atom features outside the reference vocabulary")
        a = ea[0::2]
        if a.size and (a[:, 0].min() < 0 or a[:, 0].max() >= MAX_BOND_TYPE
                       or a[:, 1].min() < 0 or a[:, 1].max() >= MAX_BOND_DIR):
            raise ValueError("bond features outside the reference vocabulary")
        xs.append(x.astype(np.uint8))
        bonds.append(fwd.T.astype(np.uint16))
        battr.append(a.astype(np.uint8))
    atom_ptr = np.concatenate([[0], np.cumsum([x.shape[0] for x in xs])]).astype(np.int64)
    bond_ptr = np.concatenate([[0], np.cumsum([b.shape[0] for b in bonds])]).astype(np.int64)
    G, Na, Nb = len(mols), int(atom_ptr[-1]), int(bond_ptr[-1])
    lay = _layout(G, Na, Nb)
    path = Path(path)
    tmp = path.with_suffix(path.suffix + ".tmp")
    with open(tmp, "wb") as f:
        f.write(_HDR.pack(MAGIC, VERSION, int(flags), G, Na, Nb))
        for name, arr in (("atom_ptr", atom_ptr), ("bond_ptr", bond_ptr),
                          ("atoms", np.concatenate(xs, 0) if xs else np.zeros((0, 2), np.uint8)),
                          ("bonds", np.concatenate(bonds, 0) if bonds else np.zeros((0, 2), np.uint16)),
                          ("battr", np.concatenate(battr, 0) if battr else np.zeros((0, 2), np.uint8))):
            f.seek(lay[name])
            f.write(np.ascontiguousarray(arr).tobytes())
        f.truncate(lay["end"])
    os.replace(tmp, path)
    return G


class GraphShard:
    """A shard opened with numpy memory maps (nothing is read until used)."""

    def __init__(self, path):
        self.path = Path(path)
        with open(self.path, "rb") as f:
            magic, version, flags, G, Na, Nb = _HDR.unpack(f.read(_HDR.size))
        if magic != MAGIC or version != VERSION:
            raise ValueError(f"{path}: not a molclr graph shard (magic {magic!r}, v{version})")
        lay = _layout(G, Na, Nb)
        if self.path.stat().st_size < lay["end"]:
            raise ValueError(f"{path}: truncated shard")
        mm = lambda name, dt, shape: np.memmap(self.path, dtype=dt, mode="r",  # noqa: E731
                                               offset=lay[name], shape=shape)
        self.num_molecules, self.num_atoms_total, self.num_bonds_total = G, Na, Nb
        self.flags = int(flags)
        self.explicit_h = bool(flags & FLAG_EXPLICIT_H)
        self.atom_ptr = mm("atom_ptr", np.int64, (G + 1,))
        self.bond_ptr = mm("bond_ptr", np.int64, (G + 1,))
        self.atoms = mm("atoms", np.uint8, (Na, 2)) if Na else np.zeros((0, 2), np.uint8)
        self.bonds = mm("bonds", np.uint16, (Nb, 2)) if Nb else np.zeros((0, 2), np.uint16)
        self.battr = mm("battr", np.uint8, (Nb, 2)) if Nb else np.zeros((0, 2), np.uint8)

    def __len__(self):
        return self.num_molecules

    def molecule(self, g: int):
        """Molecule g in the reference's tensors: x [N,2], edge_index [2,2M]
        (pairs (s,e),(e,s) in bond order), edge_attr [2M,2] (numpy int64)."""
        from .dataset import Molecule
        a0, a1 = int(self.atom_ptr[g]), int(self.atom_ptr[g + 1])
        b0, b1 = int(self.bond_ptr[g]), int(self.bond_ptr[g + 1])
        x = np.asarray(self.atoms[a0:a1], dtype=np.int64)
        b = np.asarray(self.bonds[b0:b1], dtype=np.int64)
        at = np.asarray(self.battr[b0:b1], dtype=np.int64)
        M = b.shape[0]
        ei = np.empty((2, 2 * M), dtype=np.int64)
        ei[0, 0::2], ei[1, 0::2] = b[:, 0], b[:, 1]
        ei[0, 1::2], ei[1, 1::2] = b[:, 1], b[:, 0]
        return Molecule(x, ei, np.repeat(at, 2, axis=0))

    def store_arrays(self, start: int = 0, stop: int | None = None) -> dict:
        """Molecules [start, stop) as DeviceMoleculeStore arrays (int64 numpy):
        x, atom_ptr, edge_index (local, directed pairs), edge_attr, bond_ptr."""
        stop = self.num_molecules if stop is None else stop
        a0, a1 = int(self.atom_ptr[start]), int(self.atom_ptr[stop])
        b0, b1 = int(self.bond_ptr[start]), int(self.bond_ptr[stop])
        b = np.asarray(self.bonds[b0:b1], dtype=np.int64)
        at = np.asarray(self.battr[b0:b1], dtype=np.int64)
        M = b.shape[0]
        ei = np.empty((2, 2 * M), dtype=np.int64)
        ei[0, 0::2], ei[1, 0::2] = b[:, 0], b[:, 1]
        ei[0, 1::2], ei[1, 1::2] = b[:, 1], b[:, 0]
        return {"x": np.asarray(self.atoms[a0:a1], dtype=np.int64),
                "atom_ptr": np.asarray(self.atom_ptr[start:stop + 1], dtype=np.int64) - a0,
                "edge_index": ei, "edge_attr": np.repeat(at, 2, axis=0),
                "bond_ptr": np.asarray(self.bond_ptr[start:stop + 1], dtype=np.int64) - b0}

    def device_store(self, device, start: int = 0, stop: int | None = None):
        """A DeviceMoleculeStore of molecules [start, stop) on ``device``."""
        from .augment import DeviceMoleculeStore
        a = self.store_arrays(start, stop)
        return DeviceMoleculeStore(a["x"], a["atom_ptr"], a["edge_index"], a["edge_attr"],
                                   a["bond_ptr"], device)


class ShardMoleculeDataset(torch.utils.data.Dataset):
    """MoleculeDataset over a shard: the reference's ``__getitem__ ->
    (Data_i, Data_j)`` contract (dataset/dataset.py:61-147) with the node-mask
    views drawn from ``SeedSequence([seed, rank, index, call])``."""

    def __init__(self, path, seed: int = 0, rank: int = 0):
        super().__init__()
        self.shard = GraphShard(path)
        self.seed, self.rank = seed, rank
        self._calls = 0

    def __len__(self):
        return len(self.shard)

    def __getitem__(self, index):
        from .dataset import augment_pair
        self._calls += 1
        ss = np.random.SeedSequence([self.seed, self.rank, index, self._calls])
        ri, rj = (np.random.default_rng(s) for s in ss.spawn(2))
        return augment_pair(self.shard.molecule(index), ri, rj)


def write_synthetic_shard(path, num_molecules: int, seed: int = 0, shape: str = "uniform") -> int:
    """A shard of SURVEY §8(d) synthetic molecules (dataset.random_molecule)."""
    from .dataset import random_molecule
    rng = np.random.default_rng(seed)
    return write_shard(path, (random_molecule(rng, shape) for _ in range(num_molecules)))


def read_smiles(data_path) -> list[str]:
    """dataset/dataset.py:46-53 (and the subgraph / mix modules' copies): the
    last comma-separated field of every line, read with ``csv.reader``.  Blank
    lines, on which the reference's ``row[-1]`` raises, are skipped."""
    import csv
    out = []
    with open(data_path) as f:
        for row in csv.reader(f, delimiter=","):
            if row:
                out.append(row[-1])
    return out


NUM_CHIRALITY_TAG = 3   # rows of the model's x_embedding2 (ginet_molclr.py:10)


def featurise_smiles_file(smiles_path, shard_path, limit: int | None = None,
                          add_hs: bool = False) -> tuple[int, int]:
    """``read_smiles`` + featurisation (dataset.py:61-109, with
    ``Chem.AddHs`` first when ``add_hs``: dataset_mix.py:87-88) into a shard.
    Returns (molecules written, molecules skipped).  Skipped: SMILES the
    subset parser rejects, and molecules with a chirality tag the model has
    no embedding row for (CHI_OTHER = 3: CHIRALITY_LIST has 4 entries, the
    model's x_embedding2 3 -- the reference's nn.Embedding raises an
    IndexError on such a molecule mid-training)."""
    from .smiles import featurise
    mols, skipped = [], 0
    for i, smi in enumerate(read_smiles(smiles_path)):
        if limit is not None and i >= limit:
            break
        smi = smi.strip()
        if not smi:
            continue
        try:
            m = featurise(smi, add_hs=add_hs)
        except ValueError:
            skipped += 1
            continue
        if m.x.size and int(m.x[:, 1].max()) >= NUM_CHIRALITY_TAG:
            skipped += 1
            continue
        mols.append(m)
    write_shard(shard_path, mols, flags=FLAG_EXPLICIT_H if add_hs else 0)
    return len(mols), skipped


def is_shard(path) -> bool:
    try:
        with open(path, "rb") as f:
            return f.read(len(MAGIC)) == MAGIC
    except OSError:
        return False


def cached_smiles_shard(smiles_path, add_hs: bool = False) -> Path:
    """The featurised shard of a SMILES file, built once next to it
    (``<file>.molclr.molg``, ``<file>.molclr-h.molg`` with explicit
    hydrogens) and rebuilt when the text file is newer.  With
    torch.distributed initialised, rank 0 builds it and the others wait."""
    import torch.distributed as dist
    src = Path(smiles_path)
    dst = src.with_name(src.name + (".molclr-h.molg" if add_hs else ".molclr.molg"))
    stale = not dst.exists() or dst.stat().st_mtime < src.stat().st_mtime
    dist_on = dist.is_available() and dist.is_initialized()
    if stale and (not dist_on or dist.get_rank() == 0):
        n, skipped = featurise_smiles_file(src, dst, add_hs=add_hs)
        print(f"featurised {src}: {n} molecules, {skipped} skipped -> {dst}")
    if dist_on:
        dist.barrier()
    return dst


def molecules_of(shard: GraphShard, ids: Sequence[int]):
    return [shard.molecule(int(g)) for g in ids]
