"""torch.ops.molclr.* (molclr_amd.torch_ops, SURVEY.md §8(b) operator seam)
against the product's autograd functions on the same inputs: the same
kernels, so bit-identical values and gradients."""
import pytest
import torch

import molclr_amd.torch_ops as tops
from molclr_amd import ops
from molclr_amd.data import DeviceGraph
from molclr_amd.dataset import SyntheticPairBatches

pytestmark = pytest.mark.gpu


def _batch(dev, B=48, seed=3):
    b = SyntheticPairBatches(B, seed=seed).next()[0]
    return b.to(dev)


def test_graph_build_op_matches_device_graph(dev):
    b = _batch(dev)
    got = torch.ops.molclr.graph_build(b.edge_index, b.edge_attr, b.batch, b.x.shape[0],
                                       b.num_graphs)
    ref = DeviceGraph(b.edge_index, b.edge_attr, b.x.shape[0], b.batch, b.num_graphs)
    for name, t in zip(tops._GRAPH_FIELDS, got):
        assert torch.equal(t, getattr(ref, name)), name


def test_gine_aggregate_op_and_its_gradients(dev):
    b = _batch(dev)
    gt = torch.ops.molclr.graph_build(b.edge_index, b.edge_attr, b.batch, b.x.shape[0],
                                      b.num_graphs)
    ref_graph = DeviceGraph(b.edge_index, b.edge_attr, b.x.shape[0], b.batch, b.num_graphs)
    N, D = b.x.shape[0], 64
    torch.manual_seed(0)
    h0, E1_0, E2_0 = (torch.randn(N, D, device=dev), torch.randn(5, D, device=dev),
                      torch.randn(3, D, device=dev))
    go = torch.randn(N, D, device=dev)
    outs = []
    for use_op in (True, False):
        h, E1, E2 = (t.clone().requires_grad_(True) for t in (h0, E1_0, E2_0))
        if use_op:
            y = torch.ops.molclr.gine_aggregate(h, E1, E2, *gt[:8])
        else:
            y = ops.gine_aggregate(h, E1, E2, ref_graph)
        y.backward(go)
        outs.append((y.detach(), h.grad, E1.grad, E2.grad))
    for a, c in zip(*outs):
        assert torch.equal(a, c)


def test_segment_pool_and_l2_normalize_ops(dev):
    b = _batch(dev)
    g = DeviceGraph(b.edge_index, b.edge_attr, b.x.shape[0], b.batch, b.num_graphs)
    torch.manual_seed(1)
    h0 = torch.randn(b.x.shape[0], 128, device=dev)
    res = []
    for use_op in (True, False):
        h = h0.clone().requires_grad_(True)
        if use_op:
            p = torch.ops.molclr.segment_pool(h, g.graph_ptr, 0)
            z, _ = torch.ops.molclr.l2_normalize(p, 1e-12)
        else:
            z = ops.l2_normalize(ops.segment_pool(h, g, "mean"))
        (z * torch.arange(z.numel(), device=dev).view_as(z).float()).sum().backward()
        res.append((z.detach(), h.grad))
    for a, c in zip(*res):
        assert torch.equal(a, c)


def test_nt_xent_op(dev):
    from molclr_amd.nt_xent import NTXentLoss
    torch.manual_seed(2)
    B, C = 64, 128
    a0 = torch.nn.functional.normalize(torch.randn(B, C, device=dev), dim=1)
    b0 = torch.nn.functional.normalize(a0 + 0.5 * torch.randn(B, C, device=dev), dim=1)
    res = []
    for use_op in (True, False):
        a, b = a0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
        loss = (torch.ops.molclr.nt_xent(a, b, B, 0.1, True) if use_op
                else NTXentLoss(dev, B, 0.1, True)(a, b))
        loss.backward()
        res.append((loss.detach(), a.grad, b.grad))
    assert torch.equal(res[0][0], res[1][0])
    for x, y in zip(res[0][1:], res[1][1:]):
        assert ((x - y).norm() / y.norm()).item() < 1e-6


def test_ops_refuse_cpu_tensors(dev):
    # registered for the CUDA/HIP dispatch key only: no CPU kernel
    with pytest.raises((RuntimeError, NotImplementedError)):
        torch.ops.molclr.segment_pool(torch.zeros(4, 4), torch.zeros(2, dtype=torch.int32), 0)


def _graph_tensors(b):
    return torch.ops.molclr.graph_build(b.edge_index, b.edge_attr, b.batch, b.x.shape[0],
                                        b.num_graphs)


def test_gcn_conv_op_matches_ops(dev):
    """molclr::gcn_conv (GCNConv.forward, gcn_molclr.py:62-84) against
    ops.gcn_conv: the same launches, bit-identical output and gradients
    (weight, bias, both scalar edge tables, input)."""
    b = _batch(dev)
    gt = _graph_tensors(b)
    g = DeviceGraph(b.edge_index, b.edge_attr, b.x.shape[0], b.batch, b.num_graphs)
    N, D = b.x.shape[0], 64
    torch.manual_seed(4)
    x0, W0, b0 = torch.randn(N, D, device=dev), 0.1 * torch.randn(D, D, device=dev), \
        torch.randn(D, device=dev)
    E10, E20 = torch.randn(5, 1, device=dev), torch.randn(3, 1, device=dev)
    go = torch.randn(N, D, device=dev)
    res = []
    for use_op in (True, False):
        x, W, bias, E1, E2 = (t.clone().requires_grad_(True) for t in (x0, W0, b0, E10, E20))
        if use_op:
            y, _ = torch.ops.molclr.gcn_conv(x, W, bias, E1, E2, *gt[:8])
        else:
            y = ops.gcn_conv(x, W, bias, E1, E2, g)
        y.backward(go)
        res.append((y.detach(), x.grad, W.grad, bias.grad, E1.grad, E2.grad))
    for k, (a, c) in enumerate(zip(*res)):
        assert torch.equal(a, c), k


def test_gcn_aggregate_op_vs_float64(dev):
    """molclr::gcn_aggregate (GCNConv.propagate + bias, gcn_molclr.py:79-91)
    and its backward against a float64 restatement of PyG's add aggregation
    (self loops appended last; scalar edge embedding E1[bt] + E2[bd])."""
    b = _batch(dev)
    gt = _graph_tensors(b)
    N, D = b.x.shape[0], 32
    torch.manual_seed(5)
    xw = torch.randn(N, D, device=dev, requires_grad=True)
    E1 = torch.randn(5, 1, device=dev, requires_grad=True)
    E2 = torch.randn(3, 1, device=dev, requires_grad=True)
    bias = torch.randn(D, device=dev, requires_grad=True)
    go = torch.randn(N, D, device=dev)
    y = torch.ops.molclr.gcn_aggregate(xw, E1, E2, bias, *gt[:8])
    y.backward(go)
    ei = b.edge_index.cpu()
    ea = b.edge_attr.cpu()
    loops = torch.arange(N)
    src = torch.cat([ei[0], loops])
    dst = torch.cat([ei[1], loops])
    bt = torch.cat([ea[:, 0], torch.full((N,), 4)])
    bd = torch.cat([ea[:, 1], torch.zeros(N, dtype=torch.long)])
    r = [t.detach().cpu().double().requires_grad_(True) for t in (xw, E1, E2, bias)]
    e = r[1][bt] + r[2][bd]
    ref = torch.zeros(N, D, dtype=torch.float64).index_add(0, dst, r[0][src] + e) + r[3]
    ref.backward(go.cpu().double())
    rel = lambda a, c: ((a.detach().cpu().double() - c).norm() / c.norm()).item()  # noqa: E731
    assert rel(y, ref.detach()) < 1e-6
    for got, want in ((xw.grad, r[0].grad), (E1.grad, r[1].grad), (E2.grad, r[2].grad),
                      (bias.grad, r[3].grad)):
        assert rel(got, want) < 1e-6


@pytest.mark.parametrize("M,D", [(4096, 300), (777, 64)])
def test_mlp_and_linear_ops_match_ops(dev, M, D):
    """molclr::mlp (GINEConv.mlp / out_lin: Linear -> ReLU -> Linear) and
    molclr::linear (feat_lin) against ops.gin_mlp / ops.linear: bit-identical
    values and gradients (the h3 products at the c2 width, x6 elsewhere)."""
    torch.manual_seed(6)
    x0 = torch.randn(M, D, device=dev)
    W10, b10 = 0.1 * torch.randn(2 * D, D, device=dev), torch.randn(2 * D, device=dev)
    W20, b20 = 0.1 * torch.randn(D, 2 * D, device=dev), torch.randn(D, device=dev)
    Wl0, bl0 = 0.1 * torch.randn(48, D, device=dev), torch.randn(48, device=dev)
    go, gl = torch.randn(M, D, device=dev), torch.randn(M, 48, device=dev)
    res = []
    for use_op in (True, False):
        x, W1, b1, W2, b2, Wl, bl = (t.clone().requires_grad_(True)
                                     for t in (x0, W10, b10, W20, b20, Wl0, bl0))
        if use_op:
            z = torch.ops.molclr.mlp(x, W1, b1, W2, b2)[0]
            yl = torch.ops.molclr.linear(x, Wl, bl)
        else:
            z = ops.gin_mlp(x, W1, b1, W2, b2)
            yl = ops.linear(x, Wl, bl)
        torch.autograd.backward([z, yl], [go, gl])
        res.append((z.detach(), yl.detach(), x.grad, W1.grad, b1.grad, W2.grad, b2.grad, Wl.grad,
                    bl.grad))
    for k, (a, c) in enumerate(zip(*res)):
        assert torch.equal(a, c), k


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_batch_norm_seg_op(dev, dtype):
    """molclr::batch_norm_seg (+ ReLU) over two row segments equals two
    nn.BatchNorm1d training calls (ginet_molclr.py:107, one per view,
    molclr.py:57,60) -- outputs, running statistics, num_batches_tracked --
    and bit-identical to the product's per-segment kernel path
    (ops.batch_norm on each segment, fp32); the backward's dz / dgamma /
    dbeta against the torch reference (fp32 1e-5, bf16 storage 2e-2)."""
    from molclr_amd.torch_ops import batch_norm_seg_module
    torch.manual_seed(7)
    rows, D = (1500, 1733), 96
    z0 = (torch.randn(sum(rows), D, device=dev) * 3 + 1).to(dtype)
    gy = torch.randn(sum(rows), D, device=dev)
    bn_ref = torch.nn.BatchNorm1d(D).to(dev)
    with torch.no_grad():
        bn_ref.weight.uniform_(0.5, 1.5)
        bn_ref.bias.uniform_(-0.5, 0.5)
    bn_op = torch.nn.BatchNorm1d(D).to(dev)
    bn_op.load_state_dict(bn_ref.state_dict())
    z = z0.clone().requires_grad_(True)
    y = batch_norm_seg_module(z, bn_op, rows, relu=True)
    y.float().backward(gy)
    zr = z0.float().clone().requires_grad_(True)
    yr = torch.cat([torch.relu(bn_ref(part)) for part in zr.split(list(rows))])
    yr.backward(gy)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    rel = lambda a, c: ((a.float() - c.float()).norm() / c.float().norm()).item()  # noqa: E731
    assert rel(y, yr) < tol
    assert rel(bn_op.running_mean, bn_ref.running_mean) < 1e-5
    assert rel(bn_op.running_var, bn_ref.running_var) < 1e-5
    assert int(bn_op.num_batches_tracked) == int(bn_ref.num_batches_tracked) == 2
    assert rel(z.grad, zr.grad) < tol
    assert rel(bn_op.weight.grad, bn_ref.weight.grad) < tol
    assert rel(bn_op.bias.grad, bn_ref.bias.grad) < tol
    if dtype == torch.float32:
        # one segment: the product's single-call kernel path, bit for bit
        bn_a = torch.nn.BatchNorm1d(D).to(dev)
        bn_a.load_state_dict(bn_ref.state_dict())
        bn_b = torch.nn.BatchNorm1d(D).to(dev)
        bn_b.load_state_dict(bn_ref.state_dict())
        part = z0[: rows[0]]
        a = batch_norm_seg_module(part, bn_a, [rows[0]], relu=False)
        c = ops.batch_norm(part, bn_b, relu=False)
        assert torch.equal(a, c)
        assert torch.equal(bn_a.running_var, bn_b.running_var)
    # eval mode: running statistics, nothing updated
    bn_op.eval()
    before = bn_op.running_mean.clone()
    with torch.no_grad():
        ye = batch_norm_seg_module(z0, bn_op, rows, relu=False)
        bn_ref.eval()
        assert rel(ye, bn_ref(z0.float())) < tol
    assert torch.equal(bn_op.running_mean, before)


def test_pool_op_refuses_pyg_int64_ptr(dev):
    """PyG's int64 ``ptr`` (or one past the rows) is refused, not
    read as int32."""
    h = torch.randn(10, 8, device=dev)
    with pytest.raises(ValueError):
        torch.ops.molclr.segment_pool(h, torch.tensor([0, 4, 10], device=dev), 0)
    with pytest.raises(ValueError):
        torch.ops.molclr.segment_pool(h, torch.tensor([0, 4, 11], dtype=torch.int32, device=dev), 0)
    with pytest.raises(ValueError):
        torch.ops.molclr.segment_pool_bwd(torch.randn(2, 8, device=dev),
                                          torch.tensor([0, 4, 12], dtype=torch.int32, device=dev),
                                          10, 0)
    out = torch.ops.molclr.segment_pool(h, torch.tensor([0, 4, 10], dtype=torch.int32, device=dev), 1)
    assert torch.allclose(out, torch.stack([h[:4].sum(0), h[4:].sum(0)]))


# the reference's layers rebuilt on torch.ops.molclr alone
def _gine_layer(conv, bn, h, G, seg, relu):
    from molclr_amd.torch_ops import batch_norm_seg_module
    agg = torch.ops.molclr.gine_aggregate(h, conv.edge_embedding1.weight,
                                          conv.edge_embedding2.weight, *G)
    z = torch.ops.molclr.mlp(agg, conv.mlp[0].weight, conv.mlp[0].bias, conv.mlp[2].weight,
                             conv.mlp[2].bias)[0]
    return batch_norm_seg_module(z, bn, seg, relu)


def _gcn_layer(conv, bn, h, G, seg, relu):
    from molclr_amd.torch_ops import batch_norm_seg_module
    z = torch.ops.molclr.gcn_conv(h, conv.weight, conv.bias, conv.edge_embedding1.weight,
                                  conv.edge_embedding2.weight, *G)[0]
    return batch_norm_seg_module(z, bn, seg, relu)


def _readout(model, h, graph_ptr):
    pooled = torch.ops.molclr.segment_pool(h, graph_ptr, 0)
    feat = torch.ops.molclr.linear(pooled, model.feat_lin.weight, model.feat_lin.bias)
    out = torch.ops.molclr.mlp(feat, model.out_lin[0].weight, model.out_lin[0].bias,
                               model.out_lin[2].weight, model.out_lin[2].bias)[0]
    return feat, out


@pytest.mark.parametrize("kind", ["gin", "gcn"])
def test_reference_layers_rebuilt_on_torch_ops(dev, kind):
    """GINet / GCN's forward (ginet_molclr.py:98-117, gcn_molclr.py:139-158)
    composed from torch.ops.molclr alone -- graph_build, gine_aggregate + mlp
    or gcn_conv, batch_norm_seg, segment_pool, linear, mlp -- equals the
    product model on the same batch: outputs, running statistics and every
    parameter gradient (the same kernels in the same order)."""
    import copy

    from molclr_amd.gcn_molclr import GCN
    from molclr_amd.ginet_molclr import GINet
    torch.manual_seed(8)
    model = (GINet if kind == "gin" else GCN)(3, 64, 128).to(dev)
    twin = copy.deepcopy(model)
    b = _batch(dev, B=40, seed=9)
    # product
    h_ref, out_ref = model(b)
    (h_ref.sum() + (out_ref * out_ref).sum()).backward()
    # rebuilt
    g = _graph_tensors(b)
    G, graph_ptr = g[:8], g[8]
    h = twin.x_embedding1(b.x[:, 0]) + twin.x_embedding2(b.x[:, 1])  # ginet_molclr.py:103
    layer = _gine_layer if kind == "gin" else _gcn_layer
    L = len(twin.gnns)
    for i in range(L):
        h = layer(twin.gnns[i], twin.batch_norms[i], h, G, [b.x.shape[0]], relu=i < L - 1)
    feat, out = _readout(twin, h, graph_ptr)
    (feat.sum() + (out * out).sum()).backward()
    rel = lambda a, c: ((a.double() - c.double()).norm() / c.double().norm().clamp_min(1e-30)).item()  # noqa: E731
    assert rel(feat, h_ref) < 1e-6 and rel(out, out_ref) < 1e-6
    for (n, p), q in zip(model.named_parameters(), twin.parameters()):
        if n.endswith("mlp.2.bias") or (kind == "gcn" and n.startswith("gnns.") and n.count(".") == 2
                                          and n.endswith(".bias")):
            continue  # feeds a BatchNorm: exact gradient 0, rounding noise only
        assert rel(q.grad, p.grad) < 1e-5, n
    for a, c in zip(model.buffers(), twin.buffers()):
        assert torch.equal(a, c) if not a.is_floating_point() else rel(a, c) < 1e-6
