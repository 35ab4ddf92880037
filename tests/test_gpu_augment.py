"""On-device node-mask augmentation + collate (molclr_mask_views) against the
oracle (oracle/augment_ref.py): bit-exact Batch fields, edge cases, status
flags, and the encoder on a device-built batch."""
import numpy as np
import pytest
import torch

from molclr_amd.dataset import random_molecule
from oracle.augment_ref import MASK_ATOM, mask_views, num_masked

pytestmark = pytest.mark.gpu


def _mols(n, seed=0, shape="uniform"):
    rng = np.random.default_rng(seed)
    return [random_molecule(rng, shape) for _ in range(n)]


def _same(b, ref):
    assert np.array_equal(b.x.cpu().numpy(), ref["x"])
    assert np.array_equal(b.edge_index.cpu().numpy(), ref["edge_index"])
    assert np.array_equal(b.edge_attr.cpu().numpy(), ref["edge_attr"])
    assert np.array_equal(b.batch.cpu().numpy(), ref["batch"])
    assert np.array_equal(b.ptr.cpu().numpy(), ref["ptr"])
    assert int(b.status.item()) == 0


@pytest.mark.parametrize("B,shape,seed", [(512, "uniform", 0), (64, "uniform", 7),
                                          (1024, "pubchem", 2**40 + 3)])
def test_mask_views_match_oracle(dev, B, shape, seed):
    from molclr_amd.augment import DeviceMoleculeStore
    mols = _mols(2 * B, seed=B, shape=shape)
    store = DeviceMoleculeStore.from_molecules(mols, dev)
    ids = np.random.default_rng(seed % 1000).permutation(2 * B)[:B]
    host = store.host_store()
    bi, bj = store.mask_views(ids, seed, check=True)
    ri, rj = mask_views(host, ids, seed, 0), mask_views(host, ids, seed, 1)
    _same(bi, ri)
    _same(bj, rj)
    # per molecule: exactly max(1, N//4) masked atoms (where the original was not
    # already the mask token) and 2 * (M - M//4) kept edges
    for g, mid in enumerate(ids[:50]):
        m = mols[mid]
        ka, kb = num_masked(m.num_atoms, m.num_bonds)
        p0, p1 = int(ri["ptr"][g]), int(ri["ptr"][g + 1])
        assert (bi.x[p0:p1, 0] == MASK_ATOM).sum().item() == ka
    assert bi.edge_index.shape[1] == sum(2 * (mols[i].num_bonds - mols[i].num_bonds // 4)
                                         for i in ids)


def test_mask_views_edge_cases(dev):
    from molclr_amd.augment import DeviceMoleculeStore

    class M:
        def __init__(self, n, bonds):
            self.x = np.stack([np.arange(n) % 5, np.zeros(n, np.int64)], 1).astype(np.int64)
            ei = []
            for s, e in bonds:
                ei += [(s, e), (e, s)]
            self.edge_index = np.array(ei, dtype=np.int64).reshape(-1, 2).T.copy()
            self.edge_attr = np.repeat(np.arange(len(bonds)) % 4, 2)[:, None].repeat(2, 1)

    big = M(130, [(i, i + 1) for i in range(129)] + [(0, 64), (3, 100)])  # > 64 atoms / bonds
    mols = [M(1, []), M(2, [(0, 1)]), M(4, [(0, 1), (1, 2), (2, 3)]), big]
    store = DeviceMoleculeStore.from_molecules(mols, dev)
    host = store.host_store()
    for ids in ([0, 1, 2, 3], [3, 3, 0], [2]):
        for view in (0, 1):
            _same(store.mask_view(ids, 99, view, check=True), mask_views(host, ids, 99, view))
    empty = store.mask_view(np.zeros(0, np.int64), 1, 0, check=True)
    assert empty.x.shape == (0, 2) and empty.ptr.cpu().tolist() == [0]
    with pytest.raises(IndexError):
        store.mask_view([4], 0, 0)


def test_mask_views_status_flags(dev):
    from molclr_amd import _lib
    from molclr_amd.augment import DeviceMoleculeStore
    lib = _lib.load()
    store = DeviceMoleculeStore.from_molecules(_mols(4), dev)
    i64 = dict(dtype=torch.int64, device=dev)

    def raw(ids, N, E):
        ids_d = torch.tensor(ids, **i64)
        B = len(ids)
        outs = [torch.zeros(max(N, 1), 2, **i64), torch.zeros(2, max(E, 1), **i64),
                torch.zeros(max(E, 1), 2, **i64), torch.zeros(max(N, 1), **i64),
                torch.zeros(B + 1, **i64)]
        st = torch.full((1,), -1, dtype=torch.int32, device=dev)
        wsb = lib.molclr_mask_views_workspace_bytes(B)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        rc = lib.molclr_mask_views(store.x.data_ptr(), store.atom_ptr.data_ptr(),
                                   store.edge_index.data_ptr(), store.edge_attr.data_ptr(),
                                   store.bond_ptr.data_ptr(), store.num_molecules,
                                   store.edge_index.shape[1], ids_d.data_ptr(), B, 5, 0,
                                   *[o.data_ptr() for o in outs], N, E, st.data_ptr(),
                                   ws.data_ptr(), wsb, None)
        assert rc == 0
        return int(st.item())

    n0, m0 = int(store.num_atoms[0]), int(store.num_bonds[0])
    assert raw([0], n0, 2 * (m0 - m0 // 4)) == 0
    assert raw([0], n0 + 1, 2 * (m0 - m0 // 4)) & 2   # sizes do not match the batch
    assert raw([9], 0, 0) & 1                        # molecule id out of range
    assert lib.molclr_mask_views(None, None, None, None, None, 0, 0, None, 0, 0, 2, None, None,
                                 None, None, None, 0, 0, None, None, 0, None) != 0  # bad view


def test_encoder_on_device_views_matches_host_collate(dev):
    """The encoder sees the same Batch whether the views were built on the
    device or by the oracle on the host."""
    from molclr_amd.augment import DeviceMoleculeStore
    from molclr_amd.data import Batch
    from molclr_amd.ginet_molclr import GINet
    torch.manual_seed(0)
    model = GINet(num_layer=2, emb_dim=64, feat_dim=128).to(dev)
    store = DeviceMoleculeStore.from_molecules(_mols(40, seed=5), dev)
    ids = np.arange(0, 40, 2)
    bi = store.mask_view(ids, 11, 0, check=True)
    r = mask_views(store.host_store(), ids, 11, 0)
    ref = Batch(x=torch.from_numpy(r["x"]), edge_index=torch.from_numpy(r["edge_index"]),
                edge_attr=torch.from_numpy(r["edge_attr"]), batch=torch.from_numpy(r["batch"]))
    ref.ptr = torch.from_numpy(r["ptr"])
    ref._num_graphs = len(ids)
    with torch.no_grad():
        h1, z1 = model(bi)
        h2, z2 = model(ref.to(dev))
    assert torch.equal(h1, h2) and torch.equal(z1, z2)


# ---------------------------------------------------------------------------
# subgraph-removal / mixed views (molclr_aug_views_plan / _write)
# ---------------------------------------------------------------------------
def _same_aug(b, ref, allowed_status=0):
    assert np.array_equal(b.x.cpu().numpy(), ref["x"])
    assert np.array_equal(b.edge_index.cpu().numpy(), ref["edge_index"])
    assert np.array_equal(b.edge_attr.cpu().numpy(), ref["edge_attr"])
    assert np.array_equal(b.batch.cpu().numpy(), ref["batch"])
    assert np.array_equal(b.ptr.cpu().numpy(), ref["ptr"])
    assert int(b.status.item()) & ~allowed_status == 0


@pytest.mark.parametrize("mode", ["subgraph", "mix"])
@pytest.mark.parametrize("B,shape,seed", [(512, "uniform", 0), (256, "pubchem", 2**40 + 9)])
def test_aug_views_match_oracle(dev, mode, B, shape, seed):
    """Bit-exact Batch fields against oracle/augment_ref.py (networkx's BFS
    order incl. the CPython set frontier, the G_i.edges survival rule, mix's
    extra masks)."""
    from molclr_amd.augment import DeviceMoleculeStore
    from oracle.augment_ref import AUG_MIX, AUG_SUBGRAPH, aug_views
    mols = _mols(2 * B, seed=B + 1, shape=shape)
    store = DeviceMoleculeStore.from_molecules(mols, dev)
    ids = np.random.default_rng(seed % 997).permutation(2 * B)[:B]
    host = store.host_store()
    m = AUG_SUBGRAPH if mode == "subgraph" else AUG_MIX
    bi, bj = store.aug_views(ids, seed, mode, check=True)
    _same_aug(bi, aug_views(host, ids, seed, 0, m))
    _same_aug(bj, aug_views(host, ids, seed, 1, m))


def test_aug_views_edge_cases(dev):
    """One- and two-atom molecules, a disconnected molecule whose centre
    component is smaller than the quota (the empty-frontier guard, status bit
    3), an isolated atom, and reversed bond orientations (the subgraph module's
    (start, end) survival test)."""
    from molclr_amd.augment import DeviceMoleculeStore
    from molclr_amd.dataset import Molecule
    from oracle.augment_ref import AUG_MIX, AUG_SUBGRAPH, aug_views

    def mol(n, bonds):
        x = np.stack([np.arange(n) % 7, np.zeros(n, np.int64)], 1).astype(np.int64)
        ei, ea = [], []
        for k, (s, e) in enumerate(bonds):
            ei += [(s, e), (e, s)]
            ea += [(k % 4, 0), (k % 4, 0)]
        ei = np.asarray(ei, np.int64).T.reshape(2, -1) if ei else np.zeros((2, 0), np.int64)
        ea = np.asarray(ea, np.int64).reshape(-1, 2)
        return Molecule(x=x, edge_index=ei, edge_attr=ea)

    rng = np.random.default_rng(3)
    mols = [mol(1, []), mol(2, [(0, 1)]),
            mol(12, [(0, 1), (1, 2), (3, 4), (4, 5), (5, 6), (6, 7), (7, 8), (8, 9), (9, 10),
                     (10, 11)]),                       # components {0,1,2} and {3..11}
            mol(5, [(1, 2), (2, 3), (3, 4)]),          # atom 0 isolated
            mol(9, [(4, 3), (3, 5), (0, 5), (5, 6), (2, 6), (7, 2), (8, 7), (1, 8), (0, 4)])]
    mols += [_mols(1, seed=int(s))[0] for s in rng.integers(0, 1000, 27)]
    store = DeviceMoleculeStore.from_molecules(mols, dev)
    host = store.host_store()
    ids = np.arange(len(mols))
    for m, name in ((AUG_SUBGRAPH, "subgraph"), (AUG_MIX, "mix")):
        for seed in range(6):
            for view in (0, 1):
                b = store.aug_view(ids, seed, view, name)
                ref = aug_views(host, ids, seed, view, m)
                flags = 0
                for f in ref["flags"]:
                    flags |= (8 if f["guard"] else 0) | (32 if f["centre_outside"] else 0)
                _same_aug(b, ref, allowed_status=flags)
                assert int(b.status.item()) == flags


@pytest.mark.parametrize("mode", ["subgraph", "mix"])
def test_aug_views_large_molecules(dev, mode):
    """Molecules beyond the in-LDS plan's 256 atoms / 512 bonds (the
    reference augments every molecule, dataset_subgraph.py:96-177,
    dataset_mix.py:86-217) run the same plan from a global workspace
    (molclr_aug_views_plan_big): bit-exact against the oracle, mixed in a
    batch with ordinary molecules, status clean."""
    from molclr_amd.augment import DeviceMoleculeStore
    from molclr_amd.dataset import random_molecule
    from oracle.augment_ref import AUG_MIX, AUG_SUBGRAPH, aug_views
    rng = np.random.default_rng(17)
    mols = _mols(40, seed=5)
    for n in (257, 300, 480, 700, 1200):  # 1200 atoms: ~1350 bonds
        mols.insert(int(rng.integers(0, len(mols))), random_molecule(rng, num_atoms=n))
    store = DeviceMoleculeStore.from_molecules(mols, dev)
    assert (~store.aug_capable()).sum() == 5
    host = store.host_store()
    ids = rng.permutation(len(mols))
    m = AUG_SUBGRAPH if mode == "subgraph" else AUG_MIX
    for seed in (0, 3):
        bi, bj = store.aug_views(ids, seed, mode, check=True)
        _same_aug(bi, aug_views(host, ids, seed, 0, m))
        _same_aug(bj, aug_views(host, ids, seed, 1, m))
