"""The reference's config.yaml drop-in, end to end on the GPU: MolCLR.train()
(molclr.py:69-147) for one epoch per ``aug`` mode (molclr.py:184-191), fed
from the reference's SMILES text ``data_path`` (config.yaml:27, read_smiles
dataset/dataset.py:46-53, featurised once into a cached shard) and from a
binary shard, with both views of every batch built on the device.  The views
the trainer consumed are checked bit for bit against oracle/augment_ref.py."""
import shutil
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle.augment_ref import AUG_MIX, AUG_SUBGRAPH, aug_views, mask_views

pytestmark = pytest.mark.gpu

SMILES = Path(__file__).parent / "data" / "smiles_small.txt"


def _config(aug, data_path, tmp_path, model_type="gin", fp16=False):
    return {
        "batch_size": 16, "warm_up": 0, "epochs": 1, "load_model": "None",
        "eval_every_n_epochs": 1, "save_every_n_epochs": 1, "log_every_n_steps": 1,
        "fp16_precision": fp16, "init_lr": 0.0005, "weight_decay": "1e-5", "gpu": "cuda:0",
        "model_type": model_type,
        "model": {"num_layer": 2, "emb_dim": 64, "feat_dim": 128, "drop_ratio": 0,
                  "pool": "mean"},
        "aug": aug,
        "dataset": {"num_workers": 0, "valid_size": 0.2, "data_path": str(data_path)},
        "loss": {"temperature": 0.1, "use_cosine_similarity": True},
        "log_root": str(tmp_path / "ckpt"),
    }


def _wrapper(config):
    # main()'s module choice (molclr.py:184-191)
    if config["aug"] == "node":
        from molclr_amd.dataset import MoleculeDatasetWrapper
    elif config["aug"] == "subgraph":
        from molclr_amd.dataset_subgraph import MoleculeDatasetWrapper
    else:
        from molclr_amd.dataset_mix import MoleculeDatasetWrapper
    return MoleculeDatasetWrapper(config["batch_size"], **config["dataset"])


def _same(b, ref):
    for k in ("x", "edge_index", "edge_attr", "batch", "ptr"):
        assert np.array_equal(getattr(b, k).cpu().numpy(), ref[k]), k


@pytest.mark.parametrize("source", ["smiles", "shard"])
@pytest.mark.parametrize("aug", ["node", "subgraph", "mix"])
def test_trainer_epoch_per_aug_mode(dev, tmp_path, monkeypatch, aug, source):
    from molclr_amd.molclr import MolCLR
    from molclr_amd.shards import GraphShard, featurise_smiles_file
    monkeypatch.chdir(tmp_path)
    src = tmp_path / "pubchem-small.txt"
    shutil.copy(SMILES, src)
    if source == "shard":
        data_path = tmp_path / "small.molg"
        featurise_smiles_file(src, data_path, add_hs=(aug == "mix"))
    else:
        data_path = src
    config = _config(aug, data_path, tmp_path)
    ds = _wrapper(config)
    model = MolCLR(ds, config).train()
    assert all(torch.isfinite(p).all() for p in model.parameters())
    ckpts = list((tmp_path / "ckpt").glob("*/checkpoints/model.pth"))
    assert ckpts and list((tmp_path / "ckpt").glob("*/checkpoints/model_0.pth"))
    logs = list((tmp_path / "ckpt").glob("*/scalars.jsonl"))
    if logs:  # JSONL writer (no tensorboard): the reference's tags
        tags = {line.split('"tag": "')[1].split('"')[0] for line in logs[0].read_text().splitlines()}
        assert {"train_loss", "cosine_lr_decay", "validation_loss"} <= tags

    # the views the loader builds, against the oracle on the store's host copy
    train_loader, _ = ds.get_data_loaders()
    store = train_loader.store
    if aug == "mix":  # Chem.AddHs before featurising (dataset_mix.py:87-88)
        assert (store.x[:, 0] == 0).any()
        assert GraphShard(ds.shard_path()).explicit_h
    else:
        assert not (store.x[:, 0] == 0).any()
    host = store.host_store()
    for bi, bj in train_loader:
        ids, key = train_loader.last
        for view, b in ((0, bi), (1, bj)):
            if aug == "node":
                ref = mask_views(host, ids, key, view)
            else:
                ref = aug_views(host, ids, key, view, AUG_SUBGRAPH if aug == "subgraph" else AUG_MIX)
            _same(b, ref)


def test_out_of_vocabulary_atoms_raise(dev, tmp_path, monkeypatch):
    """A chirality index the model has no row for (3 = CHI_OTHER) gives NaN
    embeddings and a status bit that check_inputs / DeviceGraph.check turn into
    an error: the reference's nn.Embedding raises IndexError there; nothing is
    clamped to a valid row."""
    from molclr_amd.data import Batch, pair_graph
    from molclr_amd.dataset import SyntheticPairBatches
    from molclr_amd.ginet_molclr import GINet
    torch.manual_seed(0)
    m = GINet(2, 64, 128).to(dev)
    xi, xj = SyntheticPairBatches(8, seed=3).next()
    x = xi.x.clone()
    x[5, 1] = 3
    bad = Batch(x=x, edge_index=xi.edge_index, edge_attr=xi.edge_attr, batch=xi.batch).to(dev)
    bad._num_graphs = 8
    xj = xj.to(dev)
    m.forward_pair(bad, xj)
    with pytest.raises(ValueError, match="embedding tables"):
        pair_graph(bad, xj).check()
    # in range: no flag
    good = xi.to(dev)
    m.forward_pair(good, xj)
    pair_graph(good, xj).check()
    # the embedding row is NaN, not a clamped valid row
    from molclr_amd import ops
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    h0 = ops.atom_embed(bad.x, m.x_embedding1.weight, m.x_embedding2.weight, st)
    assert torch.isnan(h0[5]).all() and torch.isfinite(h0[torch.arange(len(h0), device=dev) != 5]).all()
    assert int(st.item()) == 8
    # per-op path (executor off) reports the same way
    m.use_executor = False
    bad2 = Batch(x=x, edge_index=xi.edge_index, edge_attr=xi.edge_attr, batch=xi.batch).to(dev)
    bad2._num_graphs = 8
    m(bad2)
    from molclr_amd.data import device_graph
    with pytest.raises(ValueError, match="embedding tables"):
        device_graph(bad2).check()


def test_gcn_fp16_precision_trains_in_fp32(dev, tmp_path, monkeypatch):
    """model_type gcn + fp16_precision True: the reference trains it in fp32
    when apex is absent (molclr.py:14-22,93-96,121-125: a printed notice, then
    the plain backward).  Here: a RuntimeWarning, then the same fp32 training
    as fp16_precision False -- the first logged loss is bit-identical."""
    import json
    from molclr_amd.molclr import MolCLR
    monkeypatch.chdir(tmp_path)
    losses = {}
    for fp16 in (True, False):
        config = _config("node", "synthetic:64", tmp_path / str(fp16), model_type="gcn", fp16=fp16)
        torch.manual_seed(0)
        trainer = MolCLR(_wrapper(config), config)
        if fp16:
            with pytest.warns(RuntimeWarning, match="fp32"):
                model = trainer.build_model()
        else:
            model = trainer.build_model()
        assert all(p.dtype == torch.float32 for p in model.parameters())
        torch.manual_seed(0)
        out = MolCLR(_wrapper(config), config).train()
        assert all(torch.isfinite(p).all() for p in out.parameters())
        logs = list((tmp_path / str(fp16) / "ckpt").glob("*/scalars.jsonl"))
        if logs:
            losses[fp16] = [json.loads(x)["value"] for x in logs[0].read_text().splitlines()
                            if json.loads(x)["tag"] == "train_loss"]
    if losses:
        assert losses[True][0] == losses[False][0]


@pytest.mark.parametrize("aug", ["node", "subgraph"])
def test_trainer_hip_graph_matches_eager(dev, tmp_path, monkeypatch, aug):
    """``hip_graph: True`` (molclr_amd.graph_step): the epoch replays captured
    steps over the same device-built views.  The first step starts from the
    same state as the eager epoch's and logs the same loss; afterwards Adam
    amplifies rounding-level differences (the weight-gradient sums see the
    padded row count; tests/test_gpu_graph_step.py compares step by step), so
    the epochs' end states are held to a gross bound only."""
    import json
    from molclr_amd.molclr import MolCLR
    monkeypatch.chdir(tmp_path)
    out, losses = {}, {}
    for hg in (False, True):
        config = _config(aug, "synthetic:96", tmp_path / str(hg))
        config["hip_graph"] = hg
        torch.manual_seed(0)
        trainer = MolCLR(_wrapper(config), config)
        out[hg] = trainer.train()
        assert (getattr(trainer, "_captured", None) is not None) == hg
        logs = list((tmp_path / str(hg) / "ckpt").glob("*/scalars.jsonl"))
        if logs:
            losses[hg] = [json.loads(x)["value"] for x in logs[0].read_text().splitlines()
                          if json.loads(x)["tag"] == "train_loss"]
    if losses:
        assert len(losses[True]) == len(losses[False]) >= 2
        assert abs(losses[True][0] - losses[False][0]) <= 1e-6 * abs(losses[False][0])
    sd_e, sd_g = out[False].state_dict(), out[True].state_dict()
    for k, v in sd_e.items():
        a, b = sd_g[k].double(), v.double()
        assert torch.isfinite(a).all(), k
        if k.endswith("mlp.2.bias"):
            # feeds a BatchNorm: exact gradient 0, so its Adam steps follow
            # rounding noise in either run (tests/test_gpu_models.py:pre_bn_bias)
            continue
        assert (a - b).norm().item() <= 1e-2 * max(b.norm().item(), 1e-12), k


@pytest.mark.parametrize("hg", [False, True])
def test_invalid_batch_between_log_steps_raises(dev, tmp_path, monkeypatch, hg):
    """The status word is sticky: a batch with an out-of-vocabulary atom that
    is NOT the logged one (valid batches after it) still makes the next
    check_inputs raise, in the eager and in the captured step."""
    from molclr_amd.data import Batch
    from molclr_amd.dataset import SyntheticPairBatches
    from molclr_amd.molclr import MolCLR
    monkeypatch.chdir(tmp_path)
    config = _config("node", "synthetic:64", tmp_path)
    config["hip_graph"] = hg
    trainer = MolCLR(_wrapper(config), config)
    torch.manual_seed(0)
    model = trainer.build_model()
    opt, _ = trainer.build_optimizer(model)
    pairs = SyntheticPairBatches(16, seed=4).take(4)
    x = pairs[1][0].x.clone()
    x[3, 1] = 3  # CHI_OTHER: no embedding row
    xi = pairs[1][0]
    bad = Batch(x=x, edge_index=xi.edge_index, edge_attr=xi.edge_attr, batch=xi.batch)
    bad._num_graphs = 16
    pairs[1] = (bad, pairs[1][1])
    trainer.train_step(model, opt, *pairs[0], 0)
    trainer.check_inputs()  # clean so far
    for i, (a, b) in enumerate(pairs[1:]):
        trainer.train_step(model, opt, a, b, i + 1)
    assert (getattr(trainer, "_captured", None) is not None) == hg
    with pytest.raises(ValueError, match="embedding tables"):
        trainer.check_inputs()
