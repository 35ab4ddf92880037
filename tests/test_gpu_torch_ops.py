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
