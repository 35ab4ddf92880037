"""Binary graph shards and the SMILES featuriser.

The reference featurises with RDKit (dataset/dataset.py:61-109), absent here:
the featuriser is "parity unpinned" and these cases are hand-derived from the
reference's feature definitions (ATOM_LIST / CHIRALITY_LIST / BOND_LIST /
BONDDIR_LIST, dataset.py:26-43) and RDKit's documented conventions (see
molclr_amd/smiles.py)."""
import numpy as np
import pytest

from molclr_amd.dataset import MoleculeDataset, random_molecule
from molclr_amd.shards import GraphShard, ShardMoleculeDataset, featurise_smiles_file, write_shard
from molclr_amd.smiles import AROMATIC, DOUBLE, SINGLE, TRIPLE, featurise


def bonds_of(m):
    ei, ea = m.edge_index, m.edge_attr
    assert ei.shape[1] % 2 == 0
    out = []
    for k in range(ei.shape[1] // 2):
        a, b = ei[:, 2 * k]
        assert tuple(ei[:, 2 * k + 1]) == (b, a) and tuple(ea[2 * k]) == tuple(ea[2 * k + 1])
        out.append((int(a), int(b), int(ea[2 * k][0]), int(ea[2 * k][1])))
    return out


def test_simple_chains():
    m = featurise("CCO")
    assert m.x.tolist() == [[5, 0], [5, 0], [7, 0]]
    assert bonds_of(m) == [(0, 1, SINGLE, 0), (1, 2, SINGLE, 0)]
    assert bonds_of(featurise("C=O")) == [(0, 1, DOUBLE, 0)]
    assert bonds_of(featurise("C#N")) == [(0, 1, TRIPLE, 0)]
    m = featurise("CC(=O)Cl")
    assert m.x[:, 0].tolist() == [5, 5, 7, 16]
    assert bonds_of(m) == [(0, 1, SINGLE, 0), (1, 2, DOUBLE, 0), (1, 3, SINGLE, 0)]


def test_aromatic_rings_and_closure_order():
    m = featurise("c1ccccc1")
    assert m.x.tolist() == [[5, 0]] * 6
    # chain bonds in parse order, then the ring closure (opener first)
    assert bonds_of(m) == [(k, k + 1, AROMATIC, 0) for k in range(5)] + [(0, 5, AROMATIC, 0)]
    # the unmarked bond joining two aromatic rings is on no ring: SINGLE
    m = featurise("c1ccccc1c1ccccc1")
    b = bonds_of(m)
    assert b[5] == (5, 6, SINGLE, 0)
    assert sum(t == AROMATIC for *_, t, _ in b) == 12
    # closures sorted by ring number: C12CC1C2 -> (0,2) then (0,3)
    assert bonds_of(featurise("C12CC1C2"))[3:] == [(0, 2, SINGLE, 0), (0, 3, SINGLE, 0)]
    # explicit aromatic bond, pyridine nitrogen
    m = featurise("n1ccccc1")
    assert m.x[0, 0] == 6 and all(t == AROMATIC for *_, t, _ in bonds_of(m))


def test_stereo_and_hydrogens():
    assert featurise("[C@@H](F)(Cl)Br").x[0].tolist() == [5, 1]   # CW
    assert featurise("[C@H](F)(Cl)Br").x[0].tolist() == [5, 2]    # CCW
    m = featurise("F/C=C/F")
    assert [d for *_, d in bonds_of(m)] == [1, 0, 1]
    assert [d for *_, d in bonds_of(featurise("F/C=C\\F"))] == [1, 0, 2]
    assert [d for *_, d in bonds_of(featurise("C/C"))] == [0]     # no double bond next to it
    m = featurise("[H]C([H])([H])[H]")
    assert m.x.tolist() == [[5, 0]] and m.edge_index.shape == (2, 0)
    m = featurise("[Na+].[Cl-]")
    assert m.x[:, 0].tolist() == [10, 16] and m.edge_index.shape == (2, 0)
    assert featurise("[13CH4]").x.tolist() == [[5, 0]]
    assert featurise("c1cc[nH]c1").x[3, 0] == 6


@pytest.mark.parametrize("bad", ["C1CC", "*C", "C$C", "c1ccccc1(", "cC", "C((C)"])
def test_rejected_inputs(bad):
    with pytest.raises(ValueError):
        featurise(bad)


def test_shard_round_trip(tmp_path):
    rng = np.random.default_rng(0)
    mols = [random_molecule(rng) for _ in range(50)] + [featurise("c1ccccc1O"), featurise("[Na+].[Cl-]")]
    p = tmp_path / "a.molg"
    assert write_shard(p, mols) == len(mols)
    sh = GraphShard(p)
    assert len(sh) == len(mols)
    for g, m in enumerate(mols):
        r = sh.molecule(g)
        assert np.array_equal(r.x, m.x) and np.array_equal(r.edge_index, m.edge_index)
        assert np.array_equal(r.edge_attr, m.edge_attr)
    st = sh.store_arrays(3, 7)
    assert st["atom_ptr"][0] == 0 and st["atom_ptr"][-1] == st["x"].shape[0]
    assert st["edge_index"].shape[1] == 2 * st["bond_ptr"][-1]
    assert np.array_equal(st["x"][:mols[3].num_atoms], mols[3].x)
    # the dataset contract: (Data_i, Data_j) node-mask views
    ds = ShardMoleculeDataset(p, seed=1)
    a, b = ds[0]
    assert a.x.shape == tuple(mols[0].x.shape) and b.edge_index.shape[0] == 2
    assert (a.x[:, 0] == 118).sum() == max(1, mols[0].num_atoms // 4)


def test_shard_rejects_bad_input(tmp_path):
    m = random_molecule(np.random.default_rng(1))
    m.edge_attr = m.edge_attr.copy()
    m.edge_attr[1, 0] = (m.edge_attr[1, 0] + 1) % 4  # the two directions disagree
    with pytest.raises(ValueError):
        write_shard(tmp_path / "b.molg", [m])
    (tmp_path / "c.molg").write_bytes(b"NOTASHARD" + bytes(64))
    with pytest.raises(ValueError):
        GraphShard(tmp_path / "c.molg")


def test_featurise_smiles_file(tmp_path):
    src = tmp_path / "s.txt"
    src.write_text("CCO\nc1ccccc1\n*C\n\nC=O\n")
    n, skipped = featurise_smiles_file(src, tmp_path / "s.molg")
    assert (n, skipped) == (3, 1)
    assert GraphShard(tmp_path / "s.molg").molecule(1).x.shape == (6, 2)


def test_wrapper_reads_shards(tmp_path):
    from molclr_amd.dataset import MoleculeDatasetWrapper
    rng = np.random.default_rng(2)
    p = tmp_path / "w.molg"
    write_shard(p, [random_molecule(rng) for _ in range(40)])
    w = MoleculeDatasetWrapper(8, 0, 0.25, str(p), rank=0, world=1)
    tr, va = w.get_data_loaders()
    assert len(tr) == 30 // 8 and len(va) == 10 // 8
    xi, xj = next(iter(tr))
    assert xi.num_graphs == 8 and xj.num_graphs == 8


def test_sharded_sampler_disjoint_equal():
    from molclr_amd.dataset import ShardedSubsetSampler
    idx = list(range(100, 203))
    seen = []
    for r in range(4):
        s = ShardedSubsetSampler(idx, r, 4, seed=5)
        e0 = list(iter(s))
        e1 = list(iter(s))
        assert len(e0) == len(s) == 103 // 4 and e0 != e1
        seen.append(set(e0))
    assert all(not (seen[a] & seen[b]) for a in range(4) for b in range(a + 1, 4))
    assert set().union(*seen) <= set(idx)
    # rank streams of the views differ too
    ds0, ds1 = MoleculeDataset(4, seed=0, rank=0), MoleculeDataset(4, seed=0, rank=1)
    assert not np.array_equal(ds0[1][0].x.numpy(), ds1[1][0].x.numpy()) or \
        not np.array_equal(ds0[1][0].edge_index.numpy(), ds1[1][0].edge_index.numpy())
