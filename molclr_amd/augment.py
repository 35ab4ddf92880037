"""On-device node-mask augmentation + collate.

The reference builds both contrastive views of every molecule on the host in
``MoleculeDataset.__getitem__`` (dataset/dataset.py:111-147) and collates
them in the DataLoader (PyG ``Batch.from_data_list``, dataset.py:179).
:class:`DeviceMoleculeStore` keeps the un-augmented molecules resident in HBM
and produces the two collated views of a batch with ``molclr_mask_views``
(molclr_amd/csrc/augment.hip): one kernel per view, no host work beyond the
batch's molecule ids and sizes.  The returned :class:`~molclr_amd.data.Batch`
objects are what ``GINet`` / ``GCN`` take, exactly as the collated reference
batches after ``.to(device)`` (molclr.py:109-110).

Subsets follow the reference's sizes (max(1, floor(N/4)) atoms, floor(M/4)
bonds) and are uniform; they are drawn from a counter-based hash of
(seed, view, molecule id, item) instead of Python's unseeded ``random``, so
a (seed, batch) pair always gives the same views.

``aug_views(..., mode="subgraph" | "mix")`` builds the other two augmentation
modules' views the same way (dataset/dataset_subgraph.py,
dataset/dataset_mix.py; molclr_aug_views_plan / _write): the BFS subgraph
removal runs on the device, and the only host work is reading the view's edge
count between the two calls.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np
import torch

from . import _lib
from .data import Batch


class DeviceMoleculeStore:
    """Un-augmented molecules, concatenated and resident on one device.

    Fields (int64, device): ``x`` [Ntot,2]; ``atom_ptr`` [G+1];
    ``edge_index`` [2, 2Mtot] with molecule-local atom indices, every bond as
    the directed pair (s, e), (e, s) (dataset.py:93-109); ``edge_attr``
    [2Mtot, 2]; ``bond_ptr`` [G+1].  Host copies of the per-molecule atom and
    bond counts size the outputs without a device round trip.
    """

    def __init__(self, x, atom_ptr, edge_index, edge_attr, bond_ptr, device):
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("DeviceMoleculeStore needs a GPU device (no CPU path)")
        i64 = dict(dtype=torch.int64, device=device)
        self.device = device
        self.x = torch.as_tensor(x).to(**i64).contiguous()
        self.atom_ptr = torch.as_tensor(atom_ptr).to(**i64).contiguous()
        self.edge_index = torch.as_tensor(edge_index).to(**i64).contiguous()
        self.edge_attr = torch.as_tensor(edge_attr).to(**i64).contiguous()
        self.bond_ptr = torch.as_tensor(bond_ptr).to(**i64).contiguous()
        ap = np.asarray(torch.as_tensor(atom_ptr).cpu(), dtype=np.int64)
        bp = np.asarray(torch.as_tensor(bond_ptr).cpu(), dtype=np.int64)
        self.num_atoms = np.diff(ap)
        self.num_bonds = np.diff(bp)
        if self.edge_index.shape[0] != 2 or self.edge_index.shape[1] != 2 * int(bp[-1]):
            raise ValueError("edge_index must be [2, 2 * total bonds]")
        if self.edge_attr.shape != (2 * int(bp[-1]), 2) or self.x.shape != (int(ap[-1]), 2):
            raise ValueError("x / edge_attr shapes do not match atom_ptr / bond_ptr")

    @property
    def num_molecules(self) -> int:
        return int(self.num_atoms.shape[0])

    @classmethod
    def from_molecules(cls, mols: Sequence, device) -> "DeviceMoleculeStore":
        """From objects with ``x`` [N,2], ``edge_index`` [2,2M] (local),
        ``edge_attr`` [2M,2] (numpy or torch), e.g. dataset.Molecule."""
        xs = [np.asarray(m.x, dtype=np.int64) for m in mols]
        eis = [np.asarray(m.edge_index, dtype=np.int64) for m in mols]
        eas = [np.asarray(m.edge_attr, dtype=np.int64) for m in mols]
        atom_ptr = np.concatenate([[0], np.cumsum([x.shape[0] for x in xs])]).astype(np.int64)
        bond_ptr = np.concatenate([[0], np.cumsum([e.shape[1] // 2 for e in eis])]).astype(np.int64)
        return cls(np.concatenate(xs, 0), atom_ptr, np.concatenate(eis, 1),
                   np.concatenate(eas, 0), bond_ptr, device)

    def host_store(self) -> dict:
        """The store as numpy arrays (tests / oracle)."""
        return {k: getattr(self, k).cpu().numpy()
                for k in ("x", "atom_ptr", "edge_index", "edge_attr", "bond_ptr")}

    def mask_view_size(self, ids_h) -> tuple[int, int]:
        """(nodes, directed edges) of one node-masked view of the host ids:
        every atom, and the bonds left after dropping floor(M / 4) of each
        molecule's M (dataset.py:133-145) in both directions."""
        m = self.num_bonds[ids_h]
        return int(self.num_atoms[ids_h].sum()), int((2 * (m - m // 4)).sum())

    def mask_view(self, mol_ids, seed: int, view: int, check: bool = False,
                  host_ids=None) -> Batch:
        """One collated, node-masked view of the molecules ``mol_ids``.

        ``mol_ids`` may already be an int64 device tensor; give its host copy
        as ``host_ids`` to size the outputs without a device round trip."""
        on_dev = isinstance(mol_ids, torch.Tensor) and mol_ids.device == self.device
        if host_ids is None:
            host_ids = torch.as_tensor(mol_ids).cpu()
        ids_h = np.asarray(host_ids, dtype=np.int64)
        if ids_h.size and (ids_h.min() < 0 or ids_h.max() >= self.num_molecules):
            raise IndexError("molecule id out of range")
        B = int(ids_h.shape[0])
        N, E = self.mask_view_size(ids_h)
        dev = self.device
        i64 = dict(dtype=torch.int64, device=dev)
        ids = (mol_ids.to(torch.int64).contiguous() if on_dev
               else torch.as_tensor(ids_h).to(dev, non_blocking=True))
        x = torch.empty(N, 2, **i64)
        ei = torch.empty(2, E, **i64)
        ea = torch.empty(E, 2, **i64)
        batch = torch.empty(N, **i64)
        ptr = torch.empty(B + 1, **i64)
        status = torch.empty(1, dtype=torch.int32, device=dev)
        ws_bytes = _lib.query("molclr_mask_views_workspace_bytes", B)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        _lib.call("molclr_mask_views", self.x.data_ptr(), self.atom_ptr.data_ptr(),
                  self.edge_index.data_ptr(), self.edge_attr.data_ptr(), self.bond_ptr.data_ptr(),
                  self.num_molecules, int(self.edge_index.shape[1]), ids.data_ptr(), B,
                  int(seed) & 0xFFFFFFFFFFFFFFFF, int(view), x.data_ptr(), ei.data_ptr(),
                  ea.data_ptr(), batch.data_ptr(), ptr.data_ptr(), N, E, status.data_ptr(),
                  ws.data_ptr(), ws_bytes, _lib.stream_of(dev))
        if check:
            st = int(status.item())
            if st:
                raise ValueError(f"mask_views: invalid store or sizes (status {st})")
        b = Batch(x=x, edge_index=ei, edge_attr=ea, batch=batch)
        b.ptr = ptr
        b._num_graphs = B
        b.status = status
        return b

    def mask_views(self, mol_ids, seed: int, check: bool = False,
                   host_ids=None) -> tuple[Batch, Batch]:
        """(Batch_i, Batch_j): the two independent views the reference's
        ``MoleculeDataset.__getitem__`` returns, collated (dataset.py:147)."""
        return (self.mask_view(mol_ids, seed, 0, check, host_ids),
                self.mask_view(mol_ids, seed, 1, check, host_ids))

    AUG_MODES = {"subgraph": _lib.AUG_SUBGRAPH, "mix": _lib.AUG_MIX}
    AUG_MAX_ATOMS, AUG_MAX_BONDS = 256, 512   # augment.hip kAugMaxAtoms / kAugMaxBonds

    def aug_capable(self) -> np.ndarray:
        """Per molecule: small enough for the in-LDS subgraph / mix plan;
        larger ones run the same plan from a global workspace
        (molclr_aug_views_plan_big): every molecule is augmented."""
        return (self.num_atoms <= self.AUG_MAX_ATOMS) & (self.num_bonds <= self.AUG_MAX_BONDS)

    def aug_view(self, mol_ids, seed: int, view: int, mode: str = "subgraph",
                 check: bool = False, host_ids=None) -> Batch:
        """One collated subgraph-removal (dataset_subgraph.py) or mixed
        (dataset_mix.py) view of the molecules ``mol_ids``."""
        if mode not in self.AUG_MODES:
            raise ValueError(f"augmentation mode {mode!r}: subgraph or mix")
        on_dev = isinstance(mol_ids, torch.Tensor) and mol_ids.device == self.device
        if host_ids is None:
            host_ids = torch.as_tensor(mol_ids).cpu()
        ids_h = np.asarray(host_ids, dtype=np.int64)
        if ids_h.size and (ids_h.min() < 0 or ids_h.max() >= self.num_molecules):
            raise IndexError("molecule id out of range")
        B = int(ids_h.shape[0])
        N = int(self.num_atoms[ids_h].sum())
        Mb = int(self.num_bonds[ids_h].sum())
        dev = self.device
        i64 = dict(dtype=torch.int64, device=dev)
        ids = (mol_ids.to(torch.int64).contiguous() if on_dev
               else torch.as_tensor(ids_h).to(dev, non_blocking=True))
        ptr = torch.empty(B + 1, **i64)
        ne = torch.empty(1, **i64)
        status = torch.empty(1, dtype=torch.int32, device=dev)
        ws_bytes = _lib.query("molclr_aug_views_workspace_bytes", B, N, Mb)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        st = _lib.stream_of(dev)
        E_store = int(self.edge_index.shape[1])
        # molecules beyond the in-LDS caps: one global-workspace slot each
        na, nb = self.num_atoms[ids_h], self.num_bonds[ids_h]
        big = (na > self.AUG_MAX_ATOMS) | (nb > self.AUG_MAX_BONDS)
        nbig = int(big.sum())
        big_atoms = int(na[big].max()) if nbig else 0
        big_bonds = int(nb[big].max()) if nbig else 0
        bws_bytes = _lib.query("molclr_aug_views_big_workspace_bytes", nbig, big_atoms, big_bonds)
        bws = torch.empty(max(bws_bytes, 1), dtype=torch.uint8, device=dev)
        _lib.call("molclr_aug_views_plan_big", self.atom_ptr.data_ptr(),
                  self.edge_index.data_ptr(), self.bond_ptr.data_ptr(), self.num_molecules,
                  E_store, ids.data_ptr(), B, int(seed) & 0xFFFFFFFFFFFFFFFF, int(view),
                  self.AUG_MODES[mode], N, Mb, ptr.data_ptr(), ne.data_ptr(), status.data_ptr(),
                  ws.data_ptr(), ws_bytes, nbig, big_atoms, big_bonds, bws.data_ptr(), bws_bytes,
                  st)
        E = int(ne.item())  # the data-dependent edge count sizes the outputs
        x = torch.empty(N, 2, **i64)
        ei = torch.empty(2, E, **i64)
        ea = torch.empty(E, 2, **i64)
        batch = torch.empty(N, **i64)
        _lib.call("molclr_aug_views_write", self.x.data_ptr(), self.atom_ptr.data_ptr(),
                  self.edge_index.data_ptr(), self.edge_attr.data_ptr(), self.bond_ptr.data_ptr(),
                  self.num_molecules, E_store, ids.data_ptr(), B, ptr.data_ptr(), N, Mb, E,
                  x.data_ptr(), ei.data_ptr(), ea.data_ptr(), batch.data_ptr(), ws.data_ptr(),
                  ws_bytes, st)
        if check:
            sv = int(status.item())
            if sv & 0b10111:
                raise ValueError(f"aug_views: invalid store, sizes or molecule (status {sv})")
        b = Batch(x=x, edge_index=ei, edge_attr=ea, batch=batch)
        b.ptr = ptr
        b._num_graphs = B
        b.status = status
        return b

    def aug_views(self, mol_ids, seed: int, mode: str = "subgraph", check: bool = False,
                  host_ids=None) -> tuple[Batch, Batch]:
        """(Batch_i, Batch_j) of dataset_subgraph.py / dataset_mix.py's
        __getitem__ (two distinct centres per molecule), collated."""
        return (self.aug_view(mol_ids, seed, 0, mode, check, host_ids),
                self.aug_view(mol_ids, seed, 1, mode, check, host_ids))
