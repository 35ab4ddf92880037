"""Known-answer checks of the encoder oracle against independent naive
restatements of the reference semantics (models/ginet_molclr.py,
models/gcn_molclr.py, PyG 1.6.3 propagate / add_self_loops / mean pool)."""
import numpy as np
import pytest
import torch

from oracle.reference_cpu import (RefGCNConv, RefGINEConv, RefGINet, global_max_pool,
                                  global_mean_pool, add_self_loops)
from molclr_amd.data import Batch, Data


def tiny_graph():
    # 4 atoms: bonds (0,1) single, (1,2) aromatic dir 1, (2,3) double; as consecutive pairs
    bonds = [(0, 1, 0, 0), (1, 2, 3, 1), (2, 3, 1, 0)]
    row, col, attr = [], [], []
    for s, e, bt, bd in bonds:
        row += [s, e]
        col += [e, s]
        attr += [[bt, bd], [bt, bd]]
    ei = torch.tensor([row, col])
    ea = torch.tensor(attr)
    x = torch.tensor([[5, 0], [6, 1], [118, 0], [7, 2]])
    return x, ei, ea


def naive_gine_aggr(x, ei, ea, E1, E2):
    N = x.shape[0]
    out = np.zeros((N, x.shape[1]), dtype=np.float64)
    for k in range(ei.shape[1]):
        s, d = int(ei[0, k]), int(ei[1, k])
        out[d] += x[s] + E1[ea[k, 0]] + E2[ea[k, 1]]
    for i in range(N):
        out[i] += x[i] + E1[4] + E2[0]
    return out


def test_add_self_loops_appends_after_edges():
    ei = torch.tensor([[0, 1], [1, 0]])
    out = add_self_loops(ei, 3)
    assert out.tolist() == [[0, 1, 0, 1, 2], [1, 0, 0, 1, 2]]


def test_gine_conv_known_answer():
    torch.manual_seed(0)
    x, ei, ea = tiny_graph()
    D = 8
    conv = RefGINEConv(D)
    h = torch.randn(4, D)
    out = conv(h, ei, ea).detach().numpy()
    aggr = naive_gine_aggr(h.numpy().astype(np.float64), ei.numpy(), ea.numpy(),
                           conv.edge_embedding1.weight.detach().numpy().astype(np.float64),
                           conv.edge_embedding2.weight.detach().numpy().astype(np.float64))
    expect = conv.mlp(torch.from_numpy(aggr).float()).detach().numpy()
    np.testing.assert_allclose(out, expect, rtol=1e-5, atol=1e-6)


def test_gcn_conv_known_answer():
    torch.manual_seed(1)
    x, ei, ea = tiny_graph()
    D = 8
    conv = RefGCNConv(D)
    with torch.no_grad():
        conv.bias.uniform_(-1, 1)
    h = torch.randn(4, D)
    out = conv(h, ei, ea).detach().numpy().astype(np.float64)
    xw = (h @ conv.weight).detach().numpy().astype(np.float64)
    e1 = conv.edge_embedding1.weight.detach().numpy()[:, 0].astype(np.float64)
    e2 = conv.edge_embedding2.weight.detach().numpy()[:, 0].astype(np.float64)
    expect = np.zeros_like(xw)
    for k in range(ei.shape[1]):
        s, d = int(ei[0, k]), int(ei[1, k])
        expect[d] += xw[s] + e1[ea[k, 0]] + e2[ea[k, 1]]
    expect += xw + (e1[4] + e2[0])
    expect += conv.bias.detach().numpy()
    np.testing.assert_allclose(out, expect, rtol=1e-5, atol=1e-5)


def test_global_mean_pool_known_answer():
    h = torch.arange(12, dtype=torch.float32).view(6, 2)
    batch = torch.tensor([0, 0, 1, 1, 1, 3])  # graph 2 empty -> 0
    out = global_mean_pool(h, batch).numpy()
    np.testing.assert_allclose(out, [[1, 2], [6, 7], [0, 0], [10, 11]])


def test_global_max_pool_known_answer():
    """torch_scatter 2.0.6 scatter_max semantics: max per graph and column,
    0 for a graph without nodes, the gradient to the FIRST maximal node."""
    h = torch.tensor([[1., 5.], [3., 5.], [-2., -1.], [-7., -1.], [4., 0.]], requires_grad=True)
    batch = torch.tensor([0, 0, 1, 1, 3])  # graph 2 empty
    out = global_max_pool(h, batch)
    np.testing.assert_allclose(out.detach().numpy(), [[3, 5], [-2, -1], [0, 0], [4, 0]])
    out.backward(torch.tensor([[10., 20.], [30., 40.], [50., 60.], [70., 80.]]))
    # ties (5, 5) and (-1, -1): the first node takes the gradient
    np.testing.assert_allclose(h.grad.numpy(), [[0, 20], [10, 0], [30, 40], [0, 0], [70, 80]])
    # without ties it is torch's scatter_reduce amax
    hr = torch.randn(40, 8)
    b = torch.sort(torch.randint(0, 6, (40,))).values
    ref = torch.zeros(6, 8).scatter_reduce(0, b[:, None].expand(-1, 8), hr, "amax",
                                           include_self=False)
    np.testing.assert_allclose(global_max_pool(hr, b, 6).numpy(), ref.numpy())


def test_ginet_forward_shapes_and_batch_independence():
    """Each graph's output depends only on its own nodes (BN in eval mode)."""
    torch.manual_seed(0)
    x, ei, ea = tiny_graph()
    g1 = Data(x=x, edge_index=ei, edge_attr=ea)
    g2 = Data(x=x[:3], edge_index=ei[:, :4], edge_attr=ea[:4])
    model = RefGINet(num_layer=3, emb_dim=16, feat_dim=32).eval()
    b = Batch.from_data_list([g1, g2])
    h, out = model(b)
    assert h.shape == (2, 32) and out.shape == (2, 16)
    h1, _ = model(Batch.from_data_list([g1]))
    h2, _ = model(Batch.from_data_list([g2]))
    torch.testing.assert_close(h[0], h1[0])
    torch.testing.assert_close(h[1], h2[0])


def test_pretrained_checkpoint_loads_into_product_gcn():
    from pathlib import Path
    p = Path("/root/reference/ckpt/pretrained_gcn/checkpoints/model.pth")
    if not p.exists():
        pytest.skip("reference checkpoint not mounted (build container only)")
    from molclr_amd.gcn_molclr import GCN
    sd = torch.load(p, map_location="cpu", weights_only=True)
    m = GCN(num_layer=5, emb_dim=300, feat_dim=512)
    res = m.load_state_dict(sd, strict=True)
    assert not res.missing_keys and not res.unexpected_keys
