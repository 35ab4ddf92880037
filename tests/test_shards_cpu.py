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
    w = MoleculeDatasetWrapper(8, 0, 0.25, str(p), rank=0, world=1, views="host")
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


def test_add_hs_known_answers():
    """Chem.AddHs (dataset/dataset_mix.py:87-88): heavy atoms first, then each
    atom's hydrogens in atom order, bonded heavy -> H by SINGLE bonds appended
    after the original bonds; H is [0, 0]."""
    m = featurise("CCO", add_hs=True)
    assert m.x.tolist() == [[5, 0], [5, 0], [7, 0]] + [[0, 0]] * 6
    b = bonds_of(m)
    assert b[:2] == [(0, 1, SINGLE, 0), (1, 2, SINGLE, 0)]
    assert [(s, e) for s, e, *_ in b[2:]] == [(0, 3), (0, 4), (0, 5), (1, 6), (1, 7), (2, 8)]
    assert all(t == SINGLE and d == 0 for *_, t, d in b[2:])
    # implicit Hs: aromatic (benzene 1 per C, fused carbons 0), bracket counts, folded [H]
    cases = {"c1ccccc1": 6, "c1ccc2ccccc2c1": 8, "c1ccncc1": 5, "c1cc[nH]c1": 5, "C=O": 2,
             "[NH4+]": 4, "[H]C([H])([H])[H]": 4, "O=S(=O)(O)O": 2, "CS(C)(=O)=O": 6,
             "P(=O)(O)(O)O": 3, "[O-][N+](=O)c1ccccc1": 5, "[C@@H](F)(Cl)Br": 1}
    for smi, nh in cases.items():
        m = featurise(smi, add_hs=True)
        assert int((m.x[:, 0] == 0).sum()) == nh, smi
        assert m.edge_index.shape[1] == 2 * (len(bonds_of(featurise(smi))) + nh), smi
    # chirality tags stay on the heavy atoms
    assert featurise("[C@@H](F)(Cl)Br", add_hs=True).x[0].tolist() == [5, 1]
    with pytest.raises(ValueError):
        featurise("C(C)(C)(C)(C)C", add_hs=True)  # pentavalent carbon: RDKit rejects it


def test_read_smiles_is_the_reference_csv_rule(tmp_path):
    """dataset/dataset.py:46-53: csv.reader, last field of every row."""
    from molclr_amd.shards import read_smiles
    p = tmp_path / "r.txt"
    p.write_text("CCO\nid1,CCN\n\n\"a,b\",C=O\n")
    assert read_smiles(p) == ["CCO", "CCN", "C=O"]


def test_smiles_file_skips_chirality_outside_the_model(tmp_path):
    """CHI_OTHER (3) has no row in x_embedding2 (3 rows, ginet_molclr.py:10)."""
    src = tmp_path / "c.txt"
    src.write_text("CCO\nC[Si@SP1](F)(Cl)Br\nC=O\n")
    n, skipped = featurise_smiles_file(src, tmp_path / "c.molg")
    assert (n, skipped) == (2, 1)


def test_cached_smiles_shard_and_host_views(tmp_path):
    from pathlib import Path

    from molclr_amd.dataset import MoleculeDatasetWrapper
    from molclr_amd.shards import cached_smiles_shard
    src = tmp_path / "s.txt"
    src.write_text((Path(__file__).parent / "data" / "smiles_small.txt").read_text())
    p = cached_smiles_shard(src)
    ph = cached_smiles_shard(src, add_hs=True)
    assert p != ph and not GraphShard(p).explicit_h and GraphShard(ph).explicit_h
    assert len(GraphShard(p)) == len(GraphShard(ph)) == 50
    assert GraphShard(ph).num_atoms_total > GraphShard(p).num_atoms_total
    t = p.stat().st_mtime
    assert cached_smiles_shard(src) == p and p.stat().st_mtime == t  # not rebuilt
    # the reference config's data_path (a SMILES text file) on the host DataLoader
    w = MoleculeDatasetWrapper(8, 0, 0.2, str(src), rank=0, world=1, views="host")
    tr, va = w.get_data_loaders()
    assert len(tr) == 40 // 8 and len(va) == 10 // 8
    xi, xj = next(iter(tr))
    assert xi.num_graphs == 8 and xj.num_graphs == 8


def test_aug_modules_and_wrapper_arguments():
    from molclr_amd import dataset_mix, dataset_subgraph
    from molclr_amd.dataset import MoleculeDatasetWrapper, view_seed
    assert dataset_mix.MoleculeDatasetWrapper(8, 0, 0.1, "synthetic:10").aug == "mix"
    assert dataset_subgraph.MoleculeDatasetWrapper(8, 0, 0.1, "synthetic:10").aug == "subgraph"
    with pytest.raises(ValueError):   # subgraph / mix views are device-built only
        dataset_mix.MoleculeDatasetWrapper(8, 0, 0.1, "synthetic:10", views="host")
    with pytest.raises(ValueError):
        MoleculeDatasetWrapper(8, 0, 0.1, "synthetic:10", aug="edge")
    keys = {view_seed(0, r, e, b) for r in range(3) for e in range(3) for b in range(50)}
    assert len(keys) == 450 and all(0 <= k < 2**64 for k in keys)
