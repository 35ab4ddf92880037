"""Pin the oracle against the reference's own outputs (tests/golden/, made by
tests/golden/make_golden.py from /root/reference/utils/nt_xent.py)."""
import json

import numpy as np
import pytest
import torch

from oracle import ntxent_math
from oracle.reference_cpu import RefGCN, RefGINet, RefNTXentLoss

from .conftest import GOLDEN

CASES = sorted(GOLDEN.glob("ntxent_*.npz"))


def _rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def test_golden_fixtures_present():
    assert len(CASES) >= 6
    assert (GOLDEN / "pretrained_gcn_manifest.json").exists()


@pytest.mark.parametrize("path", CASES, ids=[p.stem for p in CASES])
def test_oracle_ntxent_matches_reference(path):
    d = np.load(path)
    zis = torch.from_numpy(d["zis"]).requires_grad_(True)
    zjs = torch.from_numpy(d["zjs"]).requires_grad_(True)
    crit = RefNTXentLoss("cpu", int(d["batch_size"]), float(d["temperature"]), bool(d["use_cosine"]))
    loss = crit(zis, zjs)
    loss.backward()
    assert abs(loss.item() - float(d["loss"])) <= 1e-6 * max(1.0, abs(float(d["loss"])))
    assert _rel(zis.grad, d["dzis"]) <= 1e-6
    assert _rel(zjs.grad, d["dzjs"]) <= 1e-6


@pytest.mark.parametrize("path", CASES, ids=[p.stem for p in CASES])
def test_closed_form_ntxent_matches_reference(path):
    """The algorithm the HIP kernels implement (lse + symmetric W gradient)
    reproduces the reference's loss and gradients."""
    d = np.load(path)
    loss, dzi, dzj = ntxent_math.ntxent(d["zis"], d["zjs"], float(d["temperature"]),
                                        bool(d["use_cosine"]))
    assert abs(loss - float(d["loss"])) <= 2e-6 * max(1.0, abs(float(d["loss"])))
    assert _rel(dzi, d["dzis"]) <= 1e-5
    assert _rel(dzj, d["dzjs"]) <= 1e-5


def test_checkpoint_manifest_matches_oracle_gcn():
    m = json.loads((GOLDEN / "pretrained_gcn_manifest.json").read_text())
    sd = RefGCN(num_layer=5, emb_dim=300, feat_dim=512).state_dict()
    assert {k: list(v.shape) for k, v in sd.items()} == m["keys"]


def test_checkpoint_manifest_matches_product_gcn():
    from molclr_amd.gcn_molclr import GCN
    m = json.loads((GOLDEN / "pretrained_gcn_manifest.json").read_text())
    sd = GCN(num_layer=5, emb_dim=300, feat_dim=512).state_dict()
    assert {k: list(v.shape) for k, v in sd.items()} == m["keys"]


def test_product_gin_keys_match_oracle_gin():
    from molclr_amd.ginet_molclr import GINet
    a = {k: list(v.shape) for k, v in GINet(3, 128, 512).state_dict().items()}
    b = {k: list(v.shape) for k, v in RefGINet(3, 128, 512).state_dict().items()}
    assert a == b


def test_seeded_init_matches_oracle():
    """Same parameter-creation order => same weights for the same seed."""
    from molclr_amd.gcn_molclr import GCN
    from molclr_amd.ginet_molclr import GINet
    for P, R in ((GINet, RefGINet), (GCN, RefGCN)):
        torch.manual_seed(123)
        a = P(2, 16, 32).state_dict()
        torch.manual_seed(123)
        b = R(2, 16, 32).state_dict()
        for k in b:
            assert torch.equal(a[k], b[k]), k


def test_trainable_param_counts():
    """SURVEY.md §8a a13 (probe-verified counts)."""
    from molclr_amd.gcn_molclr import GCN
    from molclr_amd.ginet_molclr import GINet

    def n(m):
        return sum(p.numel() for p in m.parameters())
    assert n(GINet(3, 128, 512)) == 677_248
    assert n(GINet(5, 300, 512)) == 2_404_196
    assert n(GINet(5, 512, 512)) == 5_995_264
    assert n(GCN(5, 300, 512)) == 1_039_236


def _gcn_fixture():
    import numpy as np
    d = np.load(GOLDEN / "gcn_pretrained_b16.npz")  # allow_pickle=False (default)
    sd = {k[2:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("w/")}
    return d, sd


def test_gcn_pretrained_fixture_is_the_shipped_checkpoint():
    """tests/golden/gcn_pretrained_b16.npz carries the reference's shipped
    pretrained_gcn weights (ckpt/pretrained_gcn/checkpoints/model.pth):
    every key / shape of the manifest, the manifest's sha256 of five tensors."""
    import hashlib
    d, sd = _gcn_fixture()
    m = json.loads((GOLDEN / "pretrained_gcn_manifest.json").read_text())
    assert {k: list(v.shape) for k, v in sd.items()} == m["keys"]
    for k, c in m["checksums"].items():
        assert hashlib.sha256(sd[k].numpy().tobytes()).hexdigest() == c["sha256"], k


def test_gcn_pretrained_fixture_oracle_outputs():
    """The fixture's h / out are the fp64 oracle's (eval mode) on its batch."""
    from molclr_amd.data import Batch
    from oracle.reference_cpu import RefGCN
    d, sd = _gcn_fixture()
    ref = RefGCN(5, 300, 512).double()
    ref.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in sd.items()})
    ref.eval()
    b = Batch(x=torch.from_numpy(d["x"]), edge_index=torch.from_numpy(d["edge_index"]),
              edge_attr=torch.from_numpy(d["edge_attr"]), batch=torch.from_numpy(d["batch"]))
    with torch.no_grad():
        h, out = ref(b)
    assert torch.equal(h, torch.from_numpy(d["h"])) and torch.equal(out, torch.from_numpy(d["out"]))
