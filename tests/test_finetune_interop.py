"""(f3) A pre-training checkpoint written by molclr_amd loads into the
reference's fine-tuning model (models/ginet_finetune.py:52-157 via
load_my_state_dict, finetune.py:247-257): every encoder tensor and feat_lin
transfer by name and shape; the projection head out_lin (pre-training only)
is skipped; the task head pred_head keeps its initialisation.  The GIN
reference checkpoint itself is absent (.MISSING_LARGE_BLOBS), so the
checkpoint is one molclr_amd writes, read back with the non-executing loader
(torch.load weights_only=True)."""
import pytest
import torch

from molclr_amd.ginet_molclr import GINet
from oracle.finetune_ref import FinetuneGCNLayout, FinetuneGINetLayout


@pytest.mark.parametrize("task,pred_n_layer,pred_act", [("classification", 2, "softplus"),
                                                         ("regression", 1, "relu")])
def test_pretrain_checkpoint_fits_finetune_model(tmp_path, task, pred_n_layer, pred_act):
    torch.manual_seed(0)
    pre = GINet(5, 300, 512)
    with torch.no_grad():  # non-default values everywhere, BN buffers included
        for p in pre.parameters():
            p.add_(torch.randn_like(p) * 0.1)
        for bn in pre.batch_norms:
            bn.running_mean.uniform_(-1, 1)
            bn.running_var.uniform_(0.5, 2)
            bn.num_batches_tracked.fill_(1234)
    path = tmp_path / "model.pth"
    torch.save(pre.state_dict(), path)  # molclr.py:148 (the trainer's checkpoint)
    sd = torch.load(path, map_location="cpu", weights_only=True)
    ft = FinetuneGINetLayout(task, 5, 300, 512, pred_n_layer, pred_act)
    head0 = {k: v.clone() for k, v in ft.state_dict().items() if k.startswith("pred_head.")}
    ft.load_my_state_dict(sd)
    own = ft.state_dict()
    enc = [k for k in sd if not k.startswith("out_lin.")]
    assert enc and all(k in own for k in enc), sorted(set(enc) - set(own))
    for k in enc:
        assert torch.equal(own[k], sd[k]), k
    assert all(k.startswith("out_lin.") for k in set(sd) - set(own))
    missing = set(own) - set(sd)
    assert missing == set(head0), missing  # only the task head is new
    for k, v in head0.items():
        assert torch.equal(own[k], v), k


@pytest.mark.parametrize("task", ["classification", "regression"])
def test_gcn_pretrain_checkpoint_fits_finetune_model(tmp_path, task):
    """models/gcn_finetune.py:94-174: a GCN pre-training checkpoint written by
    molclr_amd loads through the fine-tuning GCN's load_my_state_dict (:166):
    encoder + feat_lin transfer by name and shape, out_lin is skipped, the task
    head pred_lin keeps its initialisation.  The shipped pretrained_gcn
    checkpoint's key set (tests/golden/pretrained_gcn_manifest.json) is the
    same as molclr_amd's GCN state_dict (test_oracle_golden), so it fits too."""
    import json

    from molclr_amd.gcn_molclr import GCN
    from tests.conftest import GOLDEN
    torch.manual_seed(0)
    pre = GCN(5, 300, 512)
    with torch.no_grad():
        for p in pre.parameters():
            p.add_(torch.randn_like(p) * 0.1)
        for bn in pre.batch_norms:
            bn.running_mean.uniform_(-1, 1)
            bn.running_var.uniform_(0.5, 2)
            bn.num_batches_tracked.fill_(77)
    path = tmp_path / "model.pth"
    torch.save(pre.state_dict(), path)
    sd = torch.load(path, map_location="cpu", weights_only=True)
    ft = FinetuneGCNLayout(task, 5, 300, 512)
    head0 = {k: v.clone() for k, v in ft.state_dict().items() if k.startswith("pred_lin.")}
    ft.load_my_state_dict(sd)
    own = ft.state_dict()
    enc = [k for k in sd if not k.startswith("out_lin.")]
    assert enc and all(k in own for k in enc), sorted(set(enc) - set(own))
    for k in enc:
        assert torch.equal(own[k], sd[k]), k
    assert set(own) - set(sd) == set(head0)
    for k, v in head0.items():
        assert torch.equal(own[k], v), k
    # the shipped checkpoint's keys / shapes (manifest) all land in the layout
    man = json.loads((GOLDEN / "pretrained_gcn_manifest.json").read_text())
    shapes = {k: v for k, v in man["keys"].items() if not k.startswith("out_lin.")}
    assert len(shapes) > 20
    for k, shape in shapes.items():
        assert k in own and list(own[k].shape) == shape, k
