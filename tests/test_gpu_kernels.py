"""Per-kernel parity of the HIP path (through the C ABI) against the oracle.

Bar: integer outputs bit-exact; the GINE aggregation bit-exact (same
accumulation order as the reference CPU path); everything else fp32
norm-wise relative error <= 1e-5 (SURVEY.md §8c tolerance definition)."""
import numpy as np
import pytest
import torch

from molclr_amd import ops
from molclr_amd.data import DeviceGraph
from molclr_amd.dataset import SyntheticPairBatches
from oracle import ntxent_math
from oracle.graph_ref import graph_build
from oracle.reference_cpu import (RefNTXentLoss, add_self_loops, global_add_pool,
                                  global_max_pool, global_mean_pool, propagate_add)

from .conftest import GOLDEN

pytestmark = pytest.mark.gpu
TOL = 1e-5


def rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return (a - b).norm().item() / max(b.norm().item(), 1e-30)


def batch(B, seed=0, shape="uniform"):
    return SyntheticPairBatches(B, seed=seed, shape=shape).next()[0]


def dgraph(b, dev):
    return DeviceGraph(b.edge_index.to(dev), b.edge_attr.to(dev), b.x.shape[0], b.batch.to(dev),
                       b.num_graphs)


# ---------------------------------------------------------------------------
@pytest.mark.parametrize("B", [1, 7, 64, 512])
def test_graph_build_bit_exact(dev, B):
    b = batch(B, seed=B)
    g = dgraph(b, dev)
    g.check()
    ref = graph_build(b.edge_index.numpy(), b.edge_attr.numpy(), b.batch.numpy(), b.x.shape[0],
                      b.num_graphs)
    E = b.edge_index.shape[1]
    got = dict(rowptr=g.rowptr, col=g.col[:E], ecode=g.ecode[:E], rowptr_t=g.rowptr_t,
               col_t=g.col_t[:E], nbr=g.nbr, nbr_t=g.nbr_t, ecount=g.ecount[: 8 * b.x.shape[0]],
               graph_ptr=g.graph_ptr)
    for k, v in got.items():
        assert np.array_equal(v.cpu().numpy(), ref[k]), k


def test_graph_build_edge_cases(dev):
    # no edges at all, isolated atoms, single-atom graphs
    x = torch.tensor([[5, 0], [6, 0], [7, 0]])
    ei = torch.zeros(2, 0, dtype=torch.long)
    ea = torch.zeros(0, 2, dtype=torch.long)
    batch_v = torch.tensor([0, 1, 1])
    g = DeviceGraph(ei.to(dev), ea.to(dev), 3, batch_v.to(dev), 2)
    g.check()
    assert g.rowptr.tolist() == [0, 0, 0, 0]
    assert g.graph_ptr.tolist() == [0, 1, 3]
    ec = g.ecount.view(-1, 8).cpu()
    assert ec[:, 4].tolist() == [1, 1, 1] and ec[:, 5].tolist() == [1, 1, 1]
    # out-of-range indices are flagged, clamped, never read out of bounds
    bad = torch.tensor([[0, 9], [1, 0]])
    g = DeviceGraph(bad.to(dev), torch.tensor([[0, 0], [7, 0]]).to(dev), 3, batch_v.to(dev), 2)
    with pytest.raises(ValueError, match="edge_index out of range"):
        g.check()
    g = DeviceGraph(ei.to(dev), ea.to(dev), 3, torch.tensor([1, 0, 1]).to(dev), 2)
    with pytest.raises(ValueError, match="batch"):
        g.check()


# ---------------------------------------------------------------------------
@pytest.mark.parametrize("B,D,types", [(64, 300, "batch"), (512, 300, "batch"),
                                       (200, 100, "uniform"), (7, 64, "uniform"),
                                       (1100, 300, "carbon")])
def test_atom_embed(dev, B, D, types):
    """Embedding lookup (bit-exact) and its table gradients: partitions with
    every table row touched (uniform types), one hot row (all carbon), ragged
    row and column counts."""
    b = batch(B, 1)
    torch.manual_seed(0)
    if types == "uniform":
        b.x = torch.stack([torch.randint(0, 119, (b.x.shape[0],)),
                           torch.randint(0, 3, (b.x.shape[0],))], 1)
    elif types == "carbon":
        b.x = torch.stack([torch.full((b.x.shape[0],), 5), torch.zeros(b.x.shape[0], dtype=torch.long)], 1)
    X1 = torch.randn(119, D)
    X2 = torch.randn(3, D)
    ref = X1[b.x[:, 0]] + X2[b.x[:, 1]]
    X1d = X1.to(dev).requires_grad_(True)
    X2d = X2.to(dev).requires_grad_(True)
    h = ops.atom_embed(b.x.to(dev), X1d, X2d)
    assert torch.equal(h.cpu(), ref)
    g = torch.randn_like(ref)
    h.backward(g.to(dev))
    X1c = X1.double().requires_grad_(True)
    X2c = X2.double().requires_grad_(True)
    (X1c[b.x[:, 0]] + X2c[b.x[:, 1]]).backward(g.double())
    assert rel(X1d.grad, X1c.grad) < TOL and rel(X2d.grad, X2c.grad) < TOL
    # untouched table rows get exactly zero
    unused = torch.ones(119, dtype=torch.bool)
    unused[b.x[:, 0].unique()] = False
    assert torch.all(X1d.grad.cpu()[unused] == 0)


# (1024, 300) and (1100, 300): N > 1024 edge-table partitions x band x 8 rows
# (24 rows at D = 300), so the partition count is capped at 1024 and the
# partitions' rows are ragged (rows_per_part not a multiple of band x 8)
@pytest.mark.parametrize("B,D", [(64, 128), (512, 300), (16, 512), (1024, 300), (1100, 300)])
def test_gine_aggregate_matches_reference_order(dev, B, D):
    b = batch(B, 2)
    N = b.x.shape[0]
    torch.manual_seed(1)
    h = torch.randn(N, D)
    E1 = torch.randn(5, D)
    E2 = torch.randn(3, D)
    # oracle: PyG propagate over add_self_loops + edge embeddings (ginet_molclr.py:29-44)
    ei = add_self_loops(b.edge_index, N)
    sl = torch.zeros(N, 2, dtype=torch.long)
    sl[:, 0] = 4
    ea = torch.cat([b.edge_attr, sl], 0)
    e = E1[ea[:, 0]] + E2[ea[:, 1]]
    hr = h.clone().requires_grad_(True)
    E1r = E1.clone().requires_grad_(True)
    E2r = E2.clone().requires_grad_(True)
    er = E1r[ea[:, 0]] + E2r[ea[:, 1]]
    ref = propagate_add(hr, ei, N, lambda xj: xj + er)
    g = dgraph(b, dev)
    hd = h.to(dev).requires_grad_(True)
    E1d = E1.to(dev).requires_grad_(True)
    E2d = E2.to(dev).requires_grad_(True)
    out = ops.gine_aggregate(hd, E1d, E2d, g)
    assert torch.equal(out.detach().cpu(), ref.detach()), "GINE aggregation not bit-exact"
    go = torch.randn(N, D)
    ref.backward(go)
    out.backward(go.to(dev))
    assert rel(hd.grad, hr.grad) < TOL
    assert rel(E1d.grad, E1r.grad) < TOL and rel(E2d.grad, E2r.grad) < TOL


def hub_batch():
    """Two molecules: a 10-atom star (hub in/out degree 9 > the 4 neighbour
    slots, the CSR/CSC fallback) with a ring bond, and an isolated atom."""
    pairs = [(0, k) for k in range(1, 10)] + [(1, 2)]
    ei = []
    for a, b_ in pairs:
        ei += [(a, b_), (b_, a)]
    ei = torch.tensor(ei, dtype=torch.long).t().contiguous()
    E = ei.shape[1]
    g = torch.Generator().manual_seed(0)
    ea = torch.stack([torch.randint(0, 4, (E,), generator=g), torch.randint(0, 3, (E,), generator=g)], 1)
    x = torch.stack([torch.randint(0, 119, (11,), generator=g), torch.randint(0, 3, (11,), generator=g)], 1)
    from molclr_amd.data import Batch, Data
    return Batch.from_data_list([Data(x=x[:10], edge_index=ei, edge_attr=ea),
                                 Data(x=x[10:], edge_index=torch.zeros(2, 0, dtype=torch.long),
                                      edge_attr=torch.zeros(0, 2, dtype=torch.long))])


@pytest.mark.parametrize("D", [4, 300])
def test_gine_aggregate_high_degree(dev, D):
    b = hub_batch()
    N = b.x.shape[0]
    g = dgraph(b, dev)
    ref_g = graph_build(b.edge_index.numpy(), b.edge_attr.numpy(), b.batch.numpy(), N, b.num_graphs)
    assert np.array_equal(g.nbr.cpu().numpy(), ref_g["nbr"])
    assert np.array_equal(g.nbr_t.cpu().numpy(), ref_g["nbr_t"])
    assert (ref_g["nbr"].view(np.uint32)[0] >> 29) == 7  # hub row overflows the slots
    torch.manual_seed(3)
    h, E1, E2 = torch.randn(N, D), torch.randn(5, D), torch.randn(3, D)
    ei = add_self_loops(b.edge_index, N)
    sl = torch.zeros(N, 2, dtype=torch.long)
    sl[:, 0] = 4
    ea = torch.cat([b.edge_attr, sl], 0)
    hr = h.clone().requires_grad_(True)
    ref = propagate_add(hr, ei, N, lambda xj: xj + (E1[ea[:, 0]] + E2[ea[:, 1]]))
    hd = h.to(dev).requires_grad_(True)
    out = ops.gine_aggregate(hd, E1.to(dev), E2.to(dev), g)
    assert torch.equal(out.detach().cpu(), ref.detach())
    go = torch.randn(N, D)
    ref.backward(go)
    out.backward(go.to(dev))
    assert torch.equal(hd.grad.cpu(), hr.grad)


@pytest.mark.parametrize("B,D", [(512, 300), (64, 4), (64, 128), (16, 512)])
def test_gine_aggregate_rowmax(dev, B, D):
    """molclr_gine_aggregate_fwd_rowmax: the plain aggregation's output bit for
    bit, its row maxima as row parts (max over parts == max |row|, exactly) and
    max |out| folded into the slot -- the h3 forward's row scales."""
    from ctypes import c_void_p
    from molclr_amd import _lib
    b = batch(B, 2) if B != 16 else hub_batch()
    N = b.x.shape[0]
    g = dgraph(b, dev)
    torch.manual_seed(4)
    h, E1, E2 = torch.randn(N, D, device=dev), torch.randn(5, D, device=dev), torch.randn(3, D, device=dev)
    ref = ops.gine_aggregate(h, E1, E2, g)
    lib = _lib.load()
    st = _lib.stream_of(dev)
    Ec = torch.empty(15, D, device=dev)
    arr = lambda t: (c_void_p * 1)(t.data_ptr())  # noqa: E731
    assert lib.molclr_edge_tables_combine(1, arr(E1), arr(E2), Ec.data_ptr(), D, st) == 0
    code = lib.molclr_rowmax_layout(D)
    nbytes = lib.molclr_rowmax_bytes(N, D)
    out = torch.empty(N, D, device=dev)
    parts = torch.full((nbytes // 4,), -1.0, device=dev)
    slot = torch.zeros(ops.MAX_SLOT, device=dev)

    def row_max(buf):
        if code > 0:  # partial arrays [P][N]
            return buf.view(code, N).max(0).values
        d4 = -code  # per-wave pairs: (max of the wave's first row's piece, of the next row's)
        w = buf.view(-1, 2).cpu()
        res = torch.zeros(N)
        for r in range(N):
            for q in range((r * d4) >> 6, ((r * d4 + d4 - 1) >> 6) + 1):
                res[r] = max(res[r], w[q, 0] if (q * 64) // d4 == r else w[q, 1])
        return res.to(dev)
    assert lib.molclr_gine_aggregate_fwd_rowmax(h.data_ptr(), g.rowptr.data_ptr(), g.col.data_ptr(),
                                                g.ecode.data_ptr(), g.nbr.data_ptr(), Ec.data_ptr(),
                                                out.data_ptr(), N, D, parts.data_ptr(),
                                                slot.data_ptr(), st) == 0
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert bool((parts >= 0).all()), "a row-max entry was left unwritten"
    assert torch.equal(row_max(parts), out.abs().max(1).values)
    assert slot.max().item() == out.abs().max().item()
    # no slot (the encoder's h3 forward folds max |agg| in the lin1 GEMM)
    parts2 = torch.full((nbytes // 4,), -1.0, device=dev)
    assert lib.molclr_gine_aggregate_fwd_rowmax(h.data_ptr(), g.rowptr.data_ptr(), g.col.data_ptr(),
                                                g.ecode.data_ptr(), g.nbr.data_ptr(), Ec.data_ptr(),
                                                out.data_ptr(), N, D, parts2.data_ptr(), None,
                                                st) == 0
    torch.cuda.synchronize()
    assert torch.equal(out, ref) and torch.equal(parts2, parts)


def test_gcn_conv(dev):
    from oracle.reference_cpu import RefGCNConv
    b = batch(64, 3)
    N, D = b.x.shape[0], 128
    torch.manual_seed(2)
    conv = RefGCNConv(D)
    with torch.no_grad():
        conv.bias.uniform_(-0.5, 0.5)
    h = torch.randn(N, D, requires_grad=True)
    ref = conv(h, b.edge_index, b.edge_attr)
    go = torch.randn(N, D)
    ref.backward(go)
    W = conv.weight.detach().to(dev).requires_grad_(True)
    bias = conv.bias.detach().to(dev).requires_grad_(True)
    E1 = conv.edge_embedding1.weight.detach().to(dev).requires_grad_(True)
    E2 = conv.edge_embedding2.weight.detach().to(dev).requires_grad_(True)
    hd = h.detach().to(dev).requires_grad_(True)
    out = ops.gcn_conv(hd, W, bias, E1, E2, dgraph(b, dev))
    assert rel(out, ref) < TOL
    out.backward(go.to(dev))
    assert rel(hd.grad, h.grad) < TOL
    assert rel(W.grad, conv.weight.grad) < TOL
    assert rel(bias.grad, conv.bias.grad) < TOL
    assert rel(E1.grad, conv.edge_embedding1.weight.grad) < TOL
    assert rel(E2.grad, conv.edge_embedding2.weight.grad) < TOL


# ---------------------------------------------------------------------------
GEMM_SHAPES = [
    (1000, 600, 300), (1000, 300, 600), (300, 600, 2000), (600, 300, 15700), (64, 64, 8),
    (33, 68, 12), (512, 512, 300), (512, 256, 512), (1024, 1024, 256),
]


@pytest.fixture(params=[-1, 0, 5, 6], ids=["auto", "f32", "p6_64x64", "p6_128x64"])
def gemm_impl(request, dev):
    """Each implementation of molclr_gemm_f32 (molclr_gemm_f32_impl's argument)."""
    return request.param


@pytest.mark.parametrize("M,N,K", GEMM_SHAPES)
@pytest.mark.parametrize("ak,bk", [(0, 0), (0, 1), (1, 1), (1, 0)])
def test_gemm_layouts(dev, gemm_impl, M, N, K, ak, bk):
    torch.manual_seed(M + N + K)
    Am = torch.randn(M, K, dtype=torch.float64)
    Bm = torch.randn(K, N, dtype=torch.float64)
    ref = Am @ Bm
    A = (Am.t() if ak else Am).contiguous().float().to(dev)
    Bt = (Bm if bk else Bm.t()).contiguous().float().to(dev)
    lda = M if ak else K
    ldb = N if bk else K
    out = ops.gemm(A, Bt, M, N, K, lda, ldb, ak, bk, impl=gemm_impl)
    assert rel(out, ref) < TOL


def test_gemm_epilogues(dev, gemm_impl):
    from molclr_amd._lib import EPI_BIAS, EPI_BIAS_RELU, EPI_RELU_MASK
    torch.manual_seed(0)
    M, N, K = 777, 600, 300
    x = torch.randn(M, K)
    W = torch.randn(N, K)
    b = torch.randn(N)
    aux = torch.randn(M, N)
    y = x.double() @ W.double().t()
    xd, Wd, bd, auxd = (t.to(dev) for t in (x, W, b, aux))
    im = dict(impl=gemm_impl)
    assert rel(ops.gemm(xd, Wd, M, N, K, K, K, 0, 0, EPI_BIAS, bias=bd, **im), y + b.double()) < TOL
    assert rel(ops.gemm(xd, Wd, M, N, K, K, K, 0, 0, EPI_BIAS_RELU, bias=bd, **im),
               (y + b.double()).clamp(min=0)) < TOL
    assert rel(ops.gemm(xd, Wd, M, N, K, K, K, 0, 0, EPI_RELU_MASK, aux=auxd, **im),
               y * (aux > 0).double()) < TOL


@pytest.mark.parametrize("ak,bk", [(0, 0), (0, 1), (1, 1), (1, 0)])
def test_gemm_split_bf16_accuracy(dev, ak, bk):
    """The split-bf16 GEMMs are as accurate as the f32-input MFMA one: their
    error against float64 stays within 2x of the f32 kernel's, elementwise-
    max and norm-wise, including a long K (the weight-gradient shape)."""
    from molclr_amd import _lib
    lib = _lib.load()
    for M, N, K, positive in ((1000, 600, 300, False), (300, 600, 15700, False),
                              (1000, 600, 300, True), (300, 600, 15700, True)):
        torch.manual_seed(K)
        if positive:  # no cancellation: elementwise relative error is meaningful
            Am = torch.rand(M, K, dtype=torch.float64)
            Bm = torch.rand(K, N, dtype=torch.float64)
        else:
            Am = torch.randn(M, K, dtype=torch.float64) * torch.logspace(-3, 3, K).double()
            Bm = torch.randn(K, N, dtype=torch.float64)
        A = (Am.t() if ak else Am).contiguous().float()
        Bt = (Bm if bk else Bm.t()).contiguous().float()
        # reference on the fp32-rounded inputs: only the GEMM's own error counts
        ref = (A.double().t() if ak else A.double()) @ (Bt.double() if bk else Bt.double().t())
        errs = {}
        for impl in (0, -1, 5, 6, "bplanes", "q6"):
            if impl in ("bplanes", "q6"):
                planes = ops.weight_planes(Bt.to(dev), N, K, N if bk else K, bk)
                out = torch.empty(M, N, device=dev)
                ws_bytes = lib.molclr_gemm_f32_workspace_bytes(M, N, K)
                ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
                Ad = A.to(dev)
                rc = lib.molclr_gemm_f32_bplanes_tile(
                    Ad.data_ptr(), planes.data_ptr(), out.data_ptr(), M, N, K,
                    M if ak else K, N, ak, 0, None, None, 0, ws.data_ptr(), ws_bytes,
                    None, 9 if impl == "q6" else 0)
                assert rc == 0
                out = out.double().cpu()
            else:
                out = ops.gemm(A.to(dev), Bt.to(dev), M, N, K, M if ak else K,
                               N if bk else K, ak, bk, impl=impl).double().cpu()
            errs[impl] = (rel(out, ref), (out - ref).abs().max().item(),
                          ((out - ref).abs() / ref.abs().clamp(min=1e-30)).max().item())
        for impl in (-1, 5, 6, "bplanes", "q6"):
            assert errs[impl][0] <= 2 * errs[0][0] + 1e-9, errs
            assert errs[impl][1] <= 2 * errs[0][1] + 1e-9, errs
            if positive:
                assert errs[impl][2] <= 2 * errs[0][2], errs


@pytest.mark.parametrize("tile", [0, 5, 6, 7, 8, 9])
@pytest.mark.parametrize("M,N,K", [(1000, 600, 300), (777, 300, 600), (64, 64, 8), (33, 68, 12),
                                   (512, 256, 512), (300, 600, 2000)])
@pytest.mark.parametrize("ak,bk", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gemm_bplanes(dev, tile, M, N, K, ak, bk):
    """molclr_gemm_f32_bplanes (pre-split weight planes) against float64, all
    epilogues, both B storage orders, both A layouts and both tiles."""
    from molclr_amd._lib import EPI_BIAS, EPI_BIAS_RELU, EPI_RELU_MASK
    if ak and M % 4:
        pytest.skip("K-major A needs M % 4 == 0")
    torch.manual_seed(M * 7 + N + K)
    Am = torch.randn(M, K, dtype=torch.float64)
    Bm = torch.randn(K, N, dtype=torch.float64)
    b = torch.randn(N, dtype=torch.float64)
    aux = torch.randn(M, N)
    A = (Am.t() if ak else Am).contiguous().float().to(dev)
    W = (Bm if bk else Bm.t()).contiguous().float().to(dev)
    y = (Am.float().double()) @ (Bm.float().double())
    lda, ldb = (M if ak else K), (N if bk else K)
    bd, auxd = b.float().to(dev), aux.to(dev)
    t = dict(tile=tile)
    got = ops.gemm_w(A, W, M, N, K, lda, ldb, ak, bk, **t)
    assert rel(got, y) < TOL
    assert rel(ops.gemm_w(A, W, M, N, K, lda, ldb, ak, bk, EPI_BIAS, bias=bd, **t),
               y + b.float().double()) < TOL
    assert rel(ops.gemm_w(A, W, M, N, K, lda, ldb, ak, bk, EPI_BIAS_RELU, bias=bd, **t),
               (y + b.float().double()).clamp(min=0)) < TOL
    assert rel(ops.gemm_w(A, W, M, N, K, lda, ldb, ak, bk, EPI_RELU_MASK, aux=auxd, **t),
               y * (aux > 0).double()) < TOL
    acc = torch.randn(M, N)
    out = acc.to(dev)
    ops.gemm_w(A, W, M, N, K, lda, ldb, ak, bk, out=out, accumulate=1, **t)
    assert rel(out, y + acc.double()) < TOL
    # the cached planes follow in-place changes of the weight
    with torch.no_grad():
        W.mul_(2.0)
    assert rel(ops.gemm_w(A, W, M, N, K, lda, ldb, ak, bk, **t), 2 * y) < TOL


@pytest.mark.parametrize("rows,n_out,n_in", [(15278, 300, 600), (15278, 600, 300), (512, 512, 300),
                                             (100, 256, 512), (37, 12, 20), (1000, 30, 64)])
@pytest.mark.parametrize("acc", [0, 1])
@pytest.mark.parametrize("groups", [2, 1])
def test_linear_wgrad(dev, rows, n_out, n_in, acc, groups):
    """dW = dy^T x and db = column sums of dy in one split-bf16 GEMM (fused for
    4-aligned shapes, gemm + colsum otherwise), against float64; both K-group
    settings of the long-K weight-gradient kernel."""
    from molclr_amd import _lib
    _check_linear_wgrad(_lib.load(), dev, rows, n_out, n_in, acc, groups)


def _check_linear_wgrad(lib, dev, rows, n_out, n_in, acc, groups):
    torch.manual_seed(rows + n_out)
    dy = torch.randn(rows, n_out)
    x = torch.randn(rows, n_in)
    W0 = torch.randn(n_out, n_in)
    b0 = torch.randn(n_out)
    dW = W0.clone().to(dev)
    db = b0.clone().to(dev)
    ws_bytes = lib.molclr_linear_wgrad_workspace_bytes(rows, n_out, n_in)
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    dyd, xd = dy.to(dev), x.to(dev)
    rc = lib.molclr_linear_wgrad_groups(dyd.data_ptr(), xd.data_ptr(), dW.data_ptr(), db.data_ptr(),
                                        rows, n_out, n_in, n_out, n_in, acc, ws.data_ptr(), ws_bytes,
                                        None, groups)
    if n_out % 4:
        assert rc == -1 and b"multiples of 4" in lib.molclr_last_error()
    else:
        assert rc == 0
        refW = dy.double().t() @ x.double() + (W0.double() if acc else 0)
        refb = dy.double().sum(0) + (b0.double() if acc else 0)
        assert rel(dW, refW) < TOL
        assert rel(db, refb) < TOL
    # without db: the weight gradient alone
    dW2 = torch.empty(n_out, n_in, device=dev)
    assert lib.molclr_linear_wgrad_groups(dyd.data_ptr(), xd.data_ptr(), dW2.data_ptr(), None, rows,
                                          n_out, n_in, n_out, n_in, 0, ws.data_ptr(), ws_bytes, None,
                                          groups) == 0
    assert rel(dW2, dy.double().t() @ x.double()) < TOL


def test_colsum(dev):
    x = torch.randn(15713, 600)
    assert rel(ops.colsum(x.to(dev)), x.double().sum(0)) < TOL


# ---------------------------------------------------------------------------
@pytest.mark.parametrize("relu", [True, False])
@pytest.mark.parametrize("rows,D", [(15711, 300), (1950, 128), (7, 512)])
def test_batchnorm_train(dev, relu, rows, D):
    torch.manual_seed(rows)
    z = torch.randn(rows, D) * 3 + 1.5
    bn_ref = torch.nn.BatchNorm1d(D)
    with torch.no_grad():
        bn_ref.weight.uniform_(0.5, 1.5)
        bn_ref.bias.uniform_(-0.5, 0.5)
    bn = torch.nn.BatchNorm1d(D).to(dev)
    bn.load_state_dict(bn_ref.state_dict())
    zr = z.clone().requires_grad_(True)
    yr = bn_ref(zr)
    if relu:
        yr = torch.relu(yr)
    zd = z.to(dev).requires_grad_(True)
    yd = ops.batch_norm(zd, bn, relu)
    assert rel(yd, yr) < TOL
    assert rel(bn.running_mean, bn_ref.running_mean) < TOL
    assert rel(bn.running_var, bn_ref.running_var) < TOL
    assert int(bn.num_batches_tracked) == 1
    g = torch.randn(rows, D)
    yr.backward(g)
    yd.backward(g.to(dev))
    assert rel(zd.grad, zr.grad) < TOL
    assert rel(bn.weight.grad, bn_ref.weight.grad) < TOL
    assert rel(bn.bias.grad, bn_ref.bias.grad) < TOL


def test_batchnorm_eval(dev):
    D = 300
    bn_ref = torch.nn.BatchNorm1d(D)
    with torch.no_grad():
        bn_ref.running_mean.uniform_(-1, 1)
        bn_ref.running_var.uniform_(0.5, 2)
    bn_ref.eval()
    bn = torch.nn.BatchNorm1d(D).to(dev)
    bn.load_state_dict(bn_ref.state_dict())
    bn.eval()
    z = torch.randn(1000, D)
    with torch.no_grad():
        assert rel(ops.batch_norm(z.to(dev), bn, True), torch.relu(bn_ref(z))) < TOL


@pytest.mark.parametrize("mode", ["mean", "add"])
def test_segment_pool(dev, mode):
    b = batch(512, 4)
    N, D = b.x.shape[0], 300
    h = torch.randn(N, D, requires_grad=True)
    ref = (global_mean_pool if mode == "mean" else global_add_pool)(h, b.batch)
    hd = h.detach().to(dev).requires_grad_(True)
    out = ops.segment_pool(hd, dgraph(b, dev), mode)
    assert rel(out, ref) < TOL
    g = torch.randn_like(ref)
    ref.backward(g)
    out.backward(g.to(dev))
    assert rel(hd.grad, h.grad) < TOL


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_segment_max(dev, dtype):
    """global_max_pool: bit-exact values, gradient to the first arg-max node
    (ties forced by integer-valued embeddings), empty graphs pool to 0."""
    from molclr_amd.data import DeviceGraph
    b = batch(300, 5)
    N, D = b.x.shape[0], 64
    torch.manual_seed(5)
    h = torch.randint(-3, 4, (N, D)).float()  # many ties
    h[: N // 2] += torch.randn(N // 2, D)      # and some without
    tdt = torch.bfloat16 if dtype == "bf16" else torch.float32
    h = h.to(tdt).float().requires_grad_(True)  # values representable in the storage type
    G = int(b.num_graphs) + 2                 # two trailing graphs without nodes
    ref = global_max_pool(h, b.batch, G)
    g = DeviceGraph(b.edge_index.to(dev), b.edge_attr.to(dev), N, b.batch.to(dev), G)
    hd = h.detach().to(tdt).to(dev).requires_grad_(True)
    out = ops.segment_pool(hd, g, "max")
    assert torch.equal(out.cpu(), ref.detach())
    gr = torch.randn_like(ref)
    ref.backward(gr)
    out.backward(gr.to(dev))
    expect = h.grad.to(tdt)  # bf16: the routed gradient is stored rounded
    assert torch.equal(hd.grad.cpu(), expect)


def test_l2_normalize(dev):
    z = torch.randn(512, 256, requires_grad=True)
    ref = torch.nn.functional.normalize(z, dim=1)
    zd = z.detach().to(dev).requires_grad_(True)
    y = ops.l2_normalize(zd)
    assert rel(y, ref) < TOL
    g = torch.randn_like(ref)
    ref.backward(g)
    y.backward(g.to(dev))
    assert rel(zd.grad, z.grad) < TOL


# ---------------------------------------------------------------------------
CASES = sorted(GOLDEN.glob("ntxent_*.npz"))


@pytest.mark.parametrize("path", CASES, ids=[p.stem for p in CASES])
def test_ntxent_vs_reference_golden(dev, path):
    from molclr_amd.nt_xent import NTXentLoss
    d = np.load(path)
    zis = torch.from_numpy(d["zis"]).to(dev).requires_grad_(True)
    zjs = torch.from_numpy(d["zjs"]).to(dev).requires_grad_(True)
    crit = NTXentLoss(dev, int(d["batch_size"]), float(d["temperature"]), bool(d["use_cosine"]))
    loss = crit(zis, zjs)
    loss.backward()
    assert abs(loss.item() - float(d["loss"])) <= TOL * max(1.0, abs(float(d["loss"])))
    assert rel(zis.grad, d["dzis"]) < TOL
    assert rel(zjs.grad, d["dzjs"]) < TOL


@pytest.mark.parametrize("B,C", [(512, 256), (1024, 256), (100, 64)])
def test_ntxent_large_vs_oracle(dev, B, C):
    from molclr_amd.nt_xent import NTXentLoss
    rng = np.random.default_rng(B)
    zi = rng.standard_normal((B, C)).astype(np.float32)
    zj = (0.5 * zi + rng.standard_normal((B, C))).astype(np.float32)
    loss_ref, dzi_ref, dzj_ref = ntxent_math.ntxent(zi, zj, 0.1, True)
    zis = torch.from_numpy(zi).to(dev).requires_grad_(True)
    zjs = torch.from_numpy(zj).to(dev).requires_grad_(True)
    loss = NTXentLoss(dev, B, 0.1, True)(zis, zjs)
    loss.backward()
    assert abs(loss.item() - loss_ref) <= TOL * max(1.0, abs(loss_ref))
    assert rel(zis.grad, dzi_ref) < TOL and rel(zjs.grad, dzj_ref) < TOL


@pytest.mark.parametrize("B,C", [(512, 512), (512, 256)])
def test_ntxent_bwd_without_kept_similarity(dev, B, C):
    """The public molclr_ntxent_bwd (sim = NULL: S recomputed inside, both
    GEMMs' split-K space from one workspace of molclr_ntxent_workspace_bytes)
    against the backward that reuses the forward's S, and the fp64 oracle.
    C = 512 makes both GEMMs split K (the workspace overflowed)."""
    from molclr_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(C)
    z = rng.standard_normal((2 * B, C)).astype(np.float32)
    z /= np.linalg.norm(z, axis=1, keepdims=True)
    R = torch.from_numpy(z).to(dev)
    n = 2 * B
    gidx = torch.arange(n, dtype=torch.int32, device=dev)
    lse, lossr = torch.empty(n, device=dev), torch.empty(n, device=dev)
    wsb = lib.molclr_ntxent_workspace_bytes(n, n, C)
    # guard bytes after the workspace catch an overflow
    ws = torch.full((wsb + 4096,), 0x5A, dtype=torch.uint8, device=dev)
    simb = lib.molclr_ntxent_sim_bytes(n, n, C, -1)
    assert simb > 0
    sim = torch.empty(simb // 4, device=dev)
    st = _lib.stream_of(dev)
    assert lib.molclr_ntxent_fwd_impl(R.data_ptr(), gidx.data_ptr(), R.data_ptr(), n, n, C, B,
                                      0.1, lse.data_ptr(), lossr.data_ptr(), sim.data_ptr(),
                                      ws.data_ptr(), wsb, st, -1) == 0
    g = torch.ones(1, device=dev)
    d_kept, d_pub = torch.empty_like(R), torch.empty_like(R)
    assert lib.molclr_ntxent_bwd_impl(R.data_ptr(), gidx.data_ptr(), R.data_ptr(), lse.data_ptr(),
                                      g.data_ptr(), n, n, C, B, 0.1, sim.data_ptr(),
                                      d_kept.data_ptr(), ws.data_ptr(), wsb, st, -1) == 0
    assert lib.molclr_ntxent_bwd(R.data_ptr(), gidx.data_ptr(), R.data_ptr(), lse.data_ptr(),
                                 g.data_ptr(), n, n, C, B, 0.1, d_pub.data_ptr(), ws.data_ptr(),
                                 wsb, st) == 0
    torch.cuda.synchronize()
    assert (ws[wsb:] == 0x5A).all(), "molclr_ntxent_bwd wrote past its workspace"
    assert torch.equal(d_pub, d_kept)
    z64 = z.astype(np.float64)
    gi = np.arange(n)
    lse_ref, lr_ref = ntxent_math.rows_forward(z64, gi, z64, B, 0.1)
    assert abs(lossr.sum().item() - lr_ref.sum()) <= TOL * abs(lr_ref.sum())
    assert rel(d_pub, ntxent_math.rows_backward(z64, gi, z64, lse_ref, B, 0.1)) < TOL
    # a workspace one byte short is refused, not overrun
    assert lib.molclr_ntxent_bwd(R.data_ptr(), gidx.data_ptr(), R.data_ptr(), lse.data_ptr(),
                                 g.data_ptr(), n, n, C, B, 0.1, d_pub.data_ptr(), ws.data_ptr(),
                                 wsb - 1, st) != 0


def test_ntxent_matches_reference_module_at_b512(dev):
    """Full reference formulation (broadcast cosine + mask + CE) at the c2 batch."""
    from molclr_amd.nt_xent import NTXentLoss
    torch.manual_seed(7)
    zi = torch.nn.functional.normalize(torch.randn(512, 256), dim=1)
    zj = torch.nn.functional.normalize(zi + 0.7 * torch.randn(512, 256), dim=1)
    a = zi.clone().requires_grad_(True)
    b = zj.clone().requires_grad_(True)
    lr = RefNTXentLoss("cpu", 512, 0.1, True)(a, b)
    lr.backward()
    ad = zi.to(dev).requires_grad_(True)
    bd = zj.to(dev).requires_grad_(True)
    l = NTXentLoss(dev, 512, 0.1, True)(ad, bd)
    l.backward()
    assert abs(l.item() - lr.item()) <= TOL * abs(lr.item())
    assert rel(ad.grad, a.grad) < TOL and rel(bd.grad, b.grad) < TOL


# ---------------------------------------------------------------------------
def test_fused_adam_matches_torch_adam(dev):
    """molclr_adam_step against torch.optim.Adam on the CPU and on the GPU (the
    multi-tensor path the reference's optimizer takes there): bias corrections
    in double, lerp / addcmul / addcdiv ordering -- the trajectories stay within
    fp32 rounding over 20 steps."""
    from molclr_amd.optim import FusedAdam
    torch.manual_seed(0)
    ps = [torch.randn(300, 600), torch.randn(600), torch.randn(5, 3)]
    ref = [p.clone().requires_grad_(True) for p in ps]
    refg = [p.clone().to(dev).requires_grad_(True) for p in ps]
    mine = [torch.nn.Parameter(p.clone().to(dev)) for p in ps]
    o_ref = torch.optim.Adam(ref, 5e-4, weight_decay=1e-5)
    o_refg = torch.optim.Adam(refg, 5e-4, weight_decay=1e-5, foreach=True)
    o_mine = FusedAdam(mine, 5e-4, weight_decay=1e-5)
    for step in range(20):
        grads = [torch.randn_like(p) for p in ps]
        for o in (o_ref, o_refg, o_mine):
            o.zero_grad()
        for p, g in zip(ref, grads):
            p.grad = g.clone()
        for p, g in zip(refg, grads):
            p.grad = g.to(dev)
        for p, g in zip(mine, grads):
            p.grad.copy_(g.to(dev))
        o_ref.step()
        o_refg.step()
        o_mine.step()
    for a, b, c in zip(mine, ref, refg):
        assert rel(a.detach(), b.detach()) < TOL
        d = (a.detach() - c.detach()).abs().max().item()
        assert d <= 32 * torch.finfo(torch.float32).eps * c.detach().abs().max().item(), d
    assert o_mine.steps_taken == 20


# ---------------------------------------------------------------------------
# the paired (both views in one pass) building blocks
def test_graph_build_multi_equals_concatenated_batch(dev):
    """molclr_graph_build_multi over (view i, view j) == molclr_graph_build over
    the PyG collate of the two batches (node / graph offsets), bit for bit."""
    from molclr_amd.data import Batch, DeviceGraph
    bi, bj = SyntheticPairBatches(37, seed=3).next()
    g2 = DeviceGraph.union([(b.edge_index.to(dev), b.edge_attr.to(dev), b.batch.to(dev),
                             b.x.shape[0], b.num_graphs) for b in (bi, bj)])
    g2.check()
    Ni = bi.x.shape[0]
    cat = Batch(x=torch.cat([bi.x, bj.x]), edge_index=torch.cat([bi.edge_index, bj.edge_index + Ni], 1),
                edge_attr=torch.cat([bi.edge_attr, bj.edge_attr]),
                batch=torch.cat([bi.batch, bj.batch + bi.num_graphs]))
    g1 = DeviceGraph(cat.edge_index.to(dev), cat.edge_attr.to(dev), cat.x.shape[0],
                     cat.batch.to(dev), 74)
    E = cat.edge_index.shape[1]
    for name in ("rowptr", "rowptr_t", "nbr", "nbr_t", "ecount", "graph_ptr"):
        assert torch.equal(getattr(g1, name), getattr(g2, name)), name
    for name in ("col", "ecode", "col_t"):
        assert torch.equal(getattr(g1, name)[:E], getattr(g2, name)[:E]), name
    assert g2.segment_nodes == [Ni, bj.x.shape[0]]
    # an out-of-range index in the second segment is flagged
    bad = bj.edge_index.clone()
    bad[0, 0] = bj.x.shape[0]
    g3 = DeviceGraph.union([(bi.edge_index.to(dev), bi.edge_attr.to(dev), bi.batch.to(dev), Ni, 37),
                            (bad.to(dev), bj.edge_attr.to(dev), bj.batch.to(dev), bj.x.shape[0], 37)])
    with pytest.raises(ValueError, match="edge_index"):
        g3.check()


@pytest.mark.parametrize("rows,D", [((15300, 15256), 300), ((7, 3), 64), ((1950, 2001, 40), 128)])
def test_batchnorm_segments_equal_separate_calls(dev, rows, D):
    """Segmented BatchNorm == one call per segment, bit for bit: outputs, saved
    statistics, running statistics (updated in segment order), num_batches_tracked,
    and the backward (dz, dgamma / dbeta summed over the segments in order)."""
    import ctypes
    from molclr_amd import _lib
    lib = _lib.load()
    torch.manual_seed(sum(rows))
    N = sum(rows)
    z = (torch.randn(N, D) * 2 + 0.5).to(dev)
    dy = torch.randn(N, D).to(dev)
    gamma, beta = (torch.rand(D) + 0.5).to(dev), torch.randn(D).to(dev)
    S = len(rows)
    seg = (ctypes.c_int64 * S)(*rows)
    wsb = lib.molclr_batchnorm_seg_workspace_bytes(S, seg, D)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    rm, rv = torch.zeros(D, device=dev), torch.ones(D, device=dev)
    nbt = torch.zeros(1, dtype=torch.int64, device=dev)
    y = torch.empty(N, D, device=dev)
    sm, si = torch.empty(S, D, device=dev), torch.empty(S, D, device=dev)
    assert lib.molclr_batchnorm_seg_fwd(z.data_ptr(), gamma.data_ptr(), beta.data_ptr(), rm.data_ptr(),
                                        rv.data_ptr(), nbt.data_ptr(), y.data_ptr(), sm.data_ptr(),
                                        si.data_ptr(), S, seg, D, 0, 0.1, 1e-5, 1, 1, ws.data_ptr(),
                                        wsb, None) == 0
    dz = torch.empty(N, D, device=dev)
    dg, db = torch.empty(D, device=dev), torch.empty(D, device=dev)
    assert lib.molclr_batchnorm_seg_bwd(dy.data_ptr(), z.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                                        sm.data_ptr(), si.data_ptr(), dz.data_ptr(), dg.data_ptr(),
                                        db.data_ptr(), S, seg, D, 0, 1, 0, ws.data_ptr(), wsb,
                                        None) == 0
    # one call per segment
    rm2, rv2 = torch.zeros(D, device=dev), torch.ones(D, device=dev)
    nbt2 = torch.zeros(1, dtype=torch.int64, device=dev)
    y2, dz2 = torch.empty(N, D, device=dev), torch.empty(N, D, device=dev)
    dg2, db2 = torch.empty(D, device=dev), torch.empty(D, device=dev)
    r0 = 0
    for s, r in enumerate(rows):
        m1, i1 = torch.empty(D, device=dev), torch.empty(D, device=dev)
        w1 = lib.molclr_batchnorm_workspace_bytes(r, D)
        ws1 = torch.empty(w1, dtype=torch.uint8, device=dev)
        assert lib.molclr_batchnorm_fwd(z[r0:].data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                                        rm2.data_ptr(), rv2.data_ptr(), nbt2.data_ptr(),
                                        y2[r0:].data_ptr(), m1.data_ptr(), i1.data_ptr(), r, D, 0.1,
                                        1e-5, 1, 1, ws1.data_ptr(), w1, None) == 0
        assert torch.equal(m1, sm[s]) and torch.equal(i1, si[s])
        assert lib.molclr_batchnorm_bwd(dy[r0:].data_ptr(), z[r0:].data_ptr(), gamma.data_ptr(),
                                        beta.data_ptr(), m1.data_ptr(), i1.data_ptr(),
                                        dz2[r0:].data_ptr(), dg2.data_ptr(), db2.data_ptr(), r, D,
                                        1, int(s > 0), ws1.data_ptr(), w1, None) == 0
        r0 += r
    torch.cuda.synchronize()
    for a, b in ((y, y2), (rm, rm2), (rv, rv2), (nbt, nbt2), (dz, dz2), (dg, dg2), (db, db2)):
        assert torch.equal(a, b)
    assert int(nbt) == S


# ---------------------------------------------------------------------------
# h3 fp32 GEMMs (three fp16 MFMAs, power-of-two scaling): every tile width
# (N 64 / 128 / 160 wide), one and two in-block K groups, partial K steps,
# per-tensor and row-wise A scaling, the max / row-max outputs.  Data with
# rows spanning 12 binades (gradient-like): row-wise scaling keeps every row
# at fp32-GEMM accuracy.
H3_SHAPES = [(30556, 600, 300), (30556, 300, 600), (1500, 128, 256), (1500, 256, 128),
             (777, 64, 36), (300, 100, 20), (5, 12, 8)]


def _h3_planes(lib, W, N, K, kmajor, dev):
    import ctypes
    nb = lib.molclr_hplanes_bytes(N, K)
    buf = torch.empty(nb, dtype=torch.uint8, device=dev)
    i64 = lambda v: (ctypes.c_int64 * 1)(v)  # noqa: E731
    rc = lib.molclr_hplanes_make_batch(1, (ctypes.c_void_p * 1)(W.data_ptr()), i64(N), i64(K),
                                       i64(W.shape[1]), (ctypes.c_int * 1)(kmajor),
                                       (ctypes.c_void_p * 1)(buf.data_ptr()), ops._stream(W))
    assert rc == 0, lib.molclr_last_error()
    return buf


@pytest.mark.parametrize("N,K", [(600, 300), (300, 600), (37, 45), (256, 512), (8, 1000)])
@pytest.mark.parametrize("kmajor", [0, 1])
def test_weight_images_bit_exact(dev, N, K, kmajor):
    """The weight-image kernel (k_planes_make_tiled: an LDS tile for K-major
    weights) writes exactly the round-to-nearest splits torch computes from
    the same values: split-bf16 planes hi = bf16(B), mid = bf16(B - hi),
    lo = bf16(B - hi - mid), single and batched entry points alike; h3 planes
    fp16(B 2^sh) and fp16(B 2^sh - hi) with sh from max |B|; zero padding
    included, for both orientations and ragged sizes."""
    import ctypes
    from molclr_amd import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(N * 7 + K + kmajor)
    ld = (N if kmajor else K) + 4  # a padded leading dimension
    rows = K if kmajor else N
    Wfull = (torch.randn(rows, ld, generator=g) * torch.exp2(torch.randint(-8, 8, (rows, 1),
                                                                           generator=g).float()))
    W = Wfull.to(dev)
    B = (Wfull[:, :N] if kmajor else Wfull[:, :K].T)  # B(k, n) as [K][N]
    i64 = lambda v: (ctypes.c_int64 * 1)(v)  # noqa: E731
    st = ops._stream(W)
    # split-bf16: batched (tiled) against the single per-element kernel
    nb = lib.molclr_bplanes_bytes(N, K)
    one = torch.full((nb,), 0x5A, dtype=torch.uint8, device=dev)
    bat = torch.full((nb,), 0xA5, dtype=torch.uint8, device=dev)
    assert lib.molclr_bplanes_make(W.data_ptr(), N, K, ld, kmajor, one.data_ptr(), st) == 0
    assert lib.molclr_bplanes_make_batch(1, (ctypes.c_void_p * 1)(W.data_ptr()), i64(N), i64(K),
                                         i64(ld), (ctypes.c_int * 1)(kmajor),
                                         (ctypes.c_void_p * 1)(bat.data_ptr()), st) == 0
    torch.cuda.synchronize()
    assert torch.equal(one, bat)
    kp = (K + 31) // 32 * 32
    npad = nb // (6 * kp)
    x = torch.zeros(npad, kp)
    x[:N, :K] = B.T
    hi = x.bfloat16()
    r = x - hi.float()
    mid = r.bfloat16()
    lo = (r - mid.float()).bfloat16()
    planes = one.view(torch.int16).view(3, npad, kp).cpu()
    for q, ref in enumerate((hi, mid, lo)):
        assert torch.equal(planes[q], ref.view(torch.int16)), q
    # h3: against torch's fp16 rounding of the scaled values
    nb = lib.molclr_hplanes_bytes(N, K)
    buf = torch.full((nb,), 0x5A, dtype=torch.uint8, device=dev)
    assert lib.molclr_hplanes_make_batch(1, (ctypes.c_void_p * 1)(W.data_ptr()), i64(N), i64(K),
                                         i64(ld), (ctypes.c_int * 1)(kmajor),
                                         (ctypes.c_void_p * 1)(buf.data_ptr()), st) == 0
    torch.cuda.synchronize()
    kp = (K + 31) // 32 * 32
    npad = (nb - 2048 * 4) // (4 * kp)
    planes = buf[: 4 * npad * kp].view(torch.float16).view(2, npad, kp).cpu()
    m = B.abs().max()
    sh = min(15 - int(torch.frexp(m).exponent), 127)
    x = torch.zeros(npad, kp)
    x[:N, :K] = B.T * 2.0 ** sh
    hi = x.half()
    lo = (x - hi.float()).half()
    assert torch.equal(planes[0].view(torch.int16), hi.view(torch.int16))
    assert torch.equal(planes[1].view(torch.int16), lo.view(torch.int16))


def test_h3_images_both_orientations_one_batch(dev):
    """A batch holding both orientations of one weight (the forward's and the
    data gradient's h3 image) runs the max pass once for the pair: every
    image, max slot included, equals the one a single-image call writes."""
    import ctypes
    from molclr_amd import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(5)
    W = (torch.randn(600, 300, generator=g) * 3).to(dev)  # [n_out][n_in], ld 300
    V = torch.randn(64, 300, generator=g).to(dev)
    # (matrix, N, K, kmajor): W as B(k = in, n = out), W as B(k = out, n = in), another weight
    jobs = [(W, 600, 300, 0), (V, 64, 300, 0), (W, 300, 600, 1)]
    bufs = [torch.full((lib.molclr_hplanes_bytes(n, k),), 0x5A, dtype=torch.uint8, device=dev)
            for _, n, k, _ in jobs]
    c = len(jobs)
    st = ops._stream(W)
    assert lib.molclr_hplanes_make_batch(
        c, (ctypes.c_void_p * c)(*[m.data_ptr() for m, *_ in jobs]),
        (ctypes.c_int64 * c)(*[n for _, n, _, _ in jobs]),
        (ctypes.c_int64 * c)(*[k for _, _, k, _ in jobs]),
        (ctypes.c_int64 * c)(*[m.shape[1] for m, *_ in jobs]),
        (ctypes.c_int * c)(*[km for *_, km in jobs]),
        (ctypes.c_void_p * c)(*[b.data_ptr() for b in bufs]), st) == 0
    torch.cuda.synchronize()
    for (m, n, k, km), b in zip(jobs, bufs):
        one = _h3_planes(lib, m, n, k, km, dev)
        torch.cuda.synchronize()
        img = b.numel() - 2048 * 4  # the fp16 planes, then the max slot (64 entries, 32 floats apart)
        assert torch.equal(one[:img], b[:img]), (n, k, km)
        assert torch.equal(one[img:].view(torch.float32)[::32], b[img:].view(torch.float32)[::32])


@pytest.mark.parametrize("M,N,K", H3_SHAPES)
@pytest.mark.parametrize("rowwise", [0, 1])
@pytest.mark.parametrize("epi", [0, 2, 3])
def test_gemm_h3(dev, M, N, K, rowwise, epi):
    from molclr_amd import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g, dtype=torch.float64)
    if rowwise:
        A *= torch.pow(10.0, -12 * torch.rand(M, 1, generator=g, dtype=torch.float64))
    W = (torch.rand(N, K, generator=g, dtype=torch.float64) * 2 - 1) / K ** 0.5
    bias = torch.randn(N, generator=g, dtype=torch.float64) * 0.1
    aux = torch.randn(M, N, generator=g, dtype=torch.float64)
    ref = A @ W.t()
    if epi == 2:
        ref = (ref + bias).clamp_min(0)
    if epi == 3:
        ref = ref * (aux > 0)
    Ad, Wd = A.float().to(dev), W.float().to(dev)
    planes = _h3_planes(lib, Wd, N, K, 0, dev)
    P = int(lib.molclr_gemm_row_parts(N))
    rows = torch.zeros(2, M, device=dev)
    crow = torch.zeros(P, M, device=dev)
    slots = torch.zeros(2, 2048, device=dev)
    aout = torch.zeros(2048, device=dev)
    rc = lib.molclr_absmax_rows_f32(Ad.data_ptr(), M, K, K, rows[0].data_ptr(),
                                    slots[0].data_ptr(), 0, ops._stream(Ad))
    assert rc == 0
    C = torch.empty(M, N, device=dev)
    bd, ad = bias.float().to(dev), aux.float().to(dev)
    rc = lib.molclr_gemm_f32_h3(Ad.data_ptr(), (rows[0] if rowwise else slots[0]).data_ptr(),
                                rowwise, planes.data_ptr(), C.data_ptr(), M, N, K, K, N, epi,
                                bd.data_ptr(), ad.data_ptr(), N, None, slots[1].data_ptr(),
                                crow.data_ptr(), aout.data_ptr(), ops._stream(Ad))
    assert rc == 0, lib.molclr_last_error()
    torch.cuda.synchronize()
    # row-wise scaling: every row at fp32 accuracy (per-row relative error)
    Cc = C.double().cpu()
    if rowwise:
        err = ((Cc - ref).norm(dim=1) / ref.norm(dim=1).clamp_min(1e-300))
        err = err[ref.norm(dim=1) > 0].max().item()
    else:
        err = rel(Cc, ref)
    assert err < 2e-6, err
    assert rows[0].cpu().equal(Ad.abs().amax(1).cpu())
    assert slots[1].max().item() == C.abs().max().item()
    assert crow.amax(0).cpu().equal(C.abs().amax(1).cpu())
    assert aout.max().item() == Ad.abs().max().item()
    if epi == 3:  # the mask from bits of (aux > 0) gives the same C bit for bit
        words = (N + 31) // 32
        pos = torch.zeros(M, words * 32, dtype=torch.bool, device=dev)
        pos[:, :N] = ad > 0
        mb = ((pos.view(M, words, 32).long() << torch.arange(32, device=dev)).sum(-1)
              .remainder(1 << 32).t().contiguous())
        mb = torch.where(mb >= (1 << 31), mb - (1 << 32), mb).to(torch.int32)
        # (on the kernel the aux form takes, impl 1; the automatic choice for
        # bits may be k_gemm_bs16, whose k order differs: fp32 accuracy there)
        for impl in (1, 0):
            C2 = torch.empty_like(C)
            rc = lib.molclr_gemm_f32_h3_impl(
                Ad.data_ptr(), (rows[0] if rowwise else slots[0]).data_ptr(), rowwise,
                planes.data_ptr(), C2.data_ptr(), M, N, K, K, N, epi, None, None, 0,
                mb.data_ptr(), None, None, None, None, ops._stream(Ad), impl)
            assert rc == 0, lib.molclr_last_error()
            torch.cuda.synchronize()
            if impl == 1:
                assert torch.equal(C2, C)
            else:
                C2c = C2.double().cpu()
                if rowwise:
                    e2 = ((C2c - ref).norm(dim=1) / ref.norm(dim=1).clamp_min(1e-300))
                    e2 = e2[ref.norm(dim=1) > 0].max().item()
                else:
                    e2 = rel(C2c, ref)
                assert e2 < 2e-6, e2


@pytest.mark.parametrize("rows,n_out,n_in", [(30556, 300, 600), (1500, 256, 128), (100, 64, 12),
                                             (777, 36, 200)])
@pytest.mark.parametrize("spread", ["uniform", "rows", "cols", "binades30"])
def test_linear_wgrad_h3(dev, rows, n_out, n_in, spread):
    """h3 weight gradient dW = dy^T x (+ db) against fp64.  ``rows``: dy's rows
    (nodes) span 12 decades, as gradient rows do; ``cols``: dy's columns (the
    rows of dW, one output feature each) span 6 decades -- a feature with a
    tiny gradient must keep its precision however large the others are.
    Checked norm-wise, per row of dW, and element by element against the
    condition-aware bound |dy|^T |x| (what any reordered fp32 sum meets).
    The weight gradients scale each operand per tensor: a dy
    column far below the tensor's max keeps its lo part only down to 2^-17 of
    the max (below that the lo part is an fp16 subnormal, absolute precision
    2^-38 max |dy|), so the ``cols`` case -- whole features 10^-6 below the
    largest -- is held to the path's fp32 tolerance 1e-5 per row and element
    (measured 4.0e-6 / 2.2e-6 per row), every other case to 2e-6.
    ``binades30``: dy's rows spread over 30 binades (the per-tensor scale's
    flush region starts 17 below the max) and the result is also held to the
    reference's own arithmetic -- torch's fp32 CPU matmul of the same
    operands, measured against fp64 here: no further from fp64 than twice
    that, norm-wise and per row of dW ("f32" must not be narrower
    than the reference's fp32)."""
    from molclr_amd import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(rows + len(spread))
    dy = torch.randn(rows, n_out, generator=g, dtype=torch.float64) * 1e-6
    if spread == "rows":
        dy *= torch.pow(10.0, -12 * torch.rand(rows, 1, generator=g, dtype=torch.float64))
    if spread == "cols":
        dy *= torch.pow(10.0, -6 * torch.rand(1, n_out, generator=g, dtype=torch.float64))
    if spread == "binades30":
        dy *= torch.pow(2.0, -30 * torch.rand(rows, 1, generator=g, dtype=torch.float64))
    x = torch.randn(rows, n_in, generator=g, dtype=torch.float64)
    dyd, xd = dy.float().to(dev), x.float().to(dev)
    dW, db = wgrad_h3(lib, dyd, xd, dev)
    ref = dy.t() @ x
    Wc = dW.double().cpu()
    assert rel(dW, ref) < 2e-6
    assert rel(db, dy.sum(0)) < 2e-6
    tol = 1e-5 if spread == "cols" else 2e-6
    row_err = ((Wc - ref).norm(dim=1) / ref.norm(dim=1)).max().item()
    assert row_err < tol, row_err
    bound = dy.abs().t() @ x.abs()
    elem = ((Wc - ref).abs() / bound).max().item()
    assert elem < tol, elem
    if spread == "binades30":  # against the reference's fp32 (torch CPU sgemm)
        r32 = (dy.float().t() @ x.float()).double()
        e32 = rel(r32, ref)
        row32 = ((r32 - ref).norm(dim=1) / ref.norm(dim=1)).max().item()
        assert rel(dW, ref) <= max(2 * e32, 1e-7), (rel(dW, ref), e32)
        assert row_err <= max(2 * row32, 1e-7), (row_err, row32)


def wgrad_h3(lib, dyd, xd, dev):
    """molclr_linear_wgrad_h3 as the encoder calls it (dy^T x, bias gradient)."""
    rows, n_out = dyd.shape
    n_in = xd.shape[1]
    slots = torch.zeros(2, 2048, device=dev)
    for t, sl in ((dyd, slots[0]), (xd, slots[1])):
        assert lib.molclr_absmax_f32(t.data_ptr(), t.shape[0], t.shape[1], t.shape[1],
                                     sl.data_ptr(), 0, ops._stream(t)) == 0
    ws_b = lib.molclr_linear_wgrad_workspace_bytes(rows, n_out, n_in)
    ws = torch.empty(ws_b, dtype=torch.uint8, device=dev)
    dW = torch.zeros(n_out, n_in, device=dev)  # accumulate into zeros
    db = torch.zeros(n_out, device=dev)
    rc = lib.molclr_linear_wgrad_h3(dyd.data_ptr(), slots[0].data_ptr(), xd.data_ptr(),
                                    slots[1].data_ptr(), dW.data_ptr(), db.data_ptr(), rows, n_out,
                                    n_in, n_out, n_in, 1, ws.data_ptr(), ws_b, ops._stream(dyd))
    assert rc == 0, lib.molclr_last_error()
    torch.cuda.synchronize()
    return dW, db


@pytest.mark.parametrize("M,N,K,epi", [(30556, 600, 300, 2), (15000, 256, 128, 2), (1500, 256, 128, 2),
                                       (333, 64, 36, 0)])
def test_gemm_bplanes_max(dev, M, N, K, epi):
    """The GEMM with its max outputs equals molclr_gemm_f32_bplanes' automatic
    choice bit for bit (q6, or the small-shape fallback), and the slots hold
    max |A|, max |C| and C's row maxima."""
    from molclr_amd import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(M)
    A = (torch.randn(M, K, generator=g) * 3).to(dev)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(dev)
    b = torch.randn(N, generator=g).to(dev)
    ref = ops.gemm_w(A, W, M, N, K, K, K, False, False, epi, bias=b)  # automatic tile
    planes = ops.weight_planes(W, N, K, K, 0)
    C = torch.empty(M, N, device=dev)
    sl = torch.zeros(2, 2048, device=dev)
    rows = torch.zeros(int(lib.molclr_gemm_row_parts(N)), M, device=dev)
    ws_b = lib.molclr_gemm_f32_workspace_bytes(M, N, K)
    ws = torch.empty(max(ws_b, 1), dtype=torch.uint8, device=dev)
    words = (N + 31) // 32
    bits = torch.zeros(words, M, dtype=torch.int32, device=dev)
    rc = lib.molclr_gemm_f32_bplanes_max(A.data_ptr(), planes.data_ptr(), C.data_ptr(), M, N, K,
                                         K, N, epi, b.data_ptr(), None, 0, sl[0].data_ptr(),
                                         sl[1].data_ptr(), rows.data_ptr(), bits.data_ptr(),
                                         ws.data_ptr(), ws_b, ops._stream(A))
    assert rc == 0, lib.molclr_last_error()
    torch.cuda.synchronize()
    assert torch.equal(C, ref)
    assert sl[0].max().item() == A.abs().max().item()
    assert sl[1].max().item() == C.abs().max().item()
    assert torch.equal(rows.amax(0), C.abs().amax(1))
    # the ReLU bits: bit j of word w <-> C[:, 32 w + j] > 0
    pos = torch.zeros(M, words * 32, dtype=torch.bool, device=dev)
    pos[:, :N] = C > 0
    want = (pos.view(M, words, 32).long() << torch.arange(32, device=dev)).sum(-1).t()
    assert torch.equal(bits.long() & 0xFFFFFFFF, want & 0xFFFFFFFF)


@pytest.mark.parametrize("rows,D,relu", [((15300, 15256), 300, 1), ((1950, 2001, 40), 128, 0)])
def test_batchnorm_seg_bwd_max(dev, rows, D, relu):
    """molclr_batchnorm_seg_bwd_max: dz bit-identical to molclr_batchnorm_seg_bwd,
    plus dz's row maxima and max slot."""
    import ctypes
    from molclr_amd import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(D)
    R = sum(rows)
    z = (torch.randn(R, D, generator=g) * 2 + 0.5).to(dev)
    dy = (torch.randn(R, D, generator=g) * 1e-4).to(dev)
    gamma, beta = torch.rand(D, generator=g).to(dev), torch.randn(D, generator=g).to(dev)
    nseg = len(rows)
    sr = (ctypes.c_int64 * nseg)(*rows)
    ws_b = lib.molclr_batchnorm_seg_workspace_bytes(nseg, sr, D)
    ws = torch.empty(ws_b, dtype=torch.uint8, device=dev)
    mean = torch.empty(nseg, D, device=dev)
    inv = torch.empty(nseg, D, device=dev)
    rm, rv = torch.zeros(D, device=dev), torch.ones(D, device=dev)
    y = torch.empty(R, D, device=dev)
    st = ops._stream(z)
    assert lib.molclr_batchnorm_seg_fwd(z.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                                        rm.data_ptr(), rv.data_ptr(), None, y.data_ptr(),
                                        mean.data_ptr(), inv.data_ptr(), nseg, sr, D, 0, 0.1,
                                        1e-5, 1, relu, ws.data_ptr(), ws_b, st) == 0
    outs = []
    for fused in (0, 1):
        dz = torch.empty(R, D, device=dev)
        dg, db = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
        rmax = torch.full((lib.molclr_bn_row_parts(D), R), 7.0, device=dev)  # all overwritten
        slot = torch.zeros(2048, device=dev)
        if fused:
            rc = lib.molclr_batchnorm_seg_bwd_max(dy.data_ptr(), z.data_ptr(), gamma.data_ptr(),
                                                  beta.data_ptr(), mean.data_ptr(), inv.data_ptr(),
                                                  dz.data_ptr(), dg.data_ptr(), db.data_ptr(), nseg,
                                                  sr, D, relu, 1, rmax.data_ptr(), slot.data_ptr(),
                                                  ws.data_ptr(), ws_b, st)
        else:
            rc = lib.molclr_batchnorm_seg_bwd(dy.data_ptr(), z.data_ptr(), gamma.data_ptr(),
                                              beta.data_ptr(), mean.data_ptr(), inv.data_ptr(),
                                              dz.data_ptr(), dg.data_ptr(), db.data_ptr(), nseg, sr,
                                              D, 0, relu, 1, ws.data_ptr(), ws_b, st)
        assert rc == 0, lib.molclr_last_error()
        outs.append((dz, dg, db, rmax, slot))
    torch.cuda.synchronize()
    for a, b in zip(outs[0][:3], outs[1][:3]):
        assert torch.equal(a, b)
    dz, rmax, slot = outs[1][0], outs[1][3], outs[1][4]
    assert torch.equal(rmax.amax(0), dz.abs().amax(1))
    assert slot.max().item() == dz.abs().max().item()


@pytest.mark.parametrize("B,C,cosine", [(512, 256, True), (37, 64, True), (40, 128, False)])
def test_ntxent_pair_normalized_bit_identical(dev, B, C, cosine):
    """NTXentLoss.forward_pair_normalized(z) -- F.normalize, the [zjs; zis]
    row swap and the cosine scaling in one molclr_ntxent_prep_pair launch each
    way -- equals forward_pair(l2_normalize(z)) bit for bit: loss and dz."""
    from molclr_amd.nt_xent import NTXentLoss
    torch.manual_seed(B + C)
    z0 = torch.randn(2 * B, C, device=dev) * 3
    z0[1] = 0.0  # a zero row: the F.normalize eps branch
    crit = NTXentLoss(dev, B, 0.1, cosine)
    za = z0.clone().requires_grad_(True)
    zb = z0.clone().requires_grad_(True)
    la = crit.forward_pair(ops.l2_normalize(za))
    la.backward()
    lb = crit.forward_pair_normalized(zb)
    lb.backward()
    assert torch.equal(la, lb)
    assert torch.equal(za.grad, zb.grad)


@pytest.mark.parametrize("rows,D", [(30556, 300), (2048, 64)])
def test_linear_wgrad_h3_pair_matches_two_calls(dev, rows, D):
    """molclr_linear_wgrad_h3_pair (the GIN layer's dW2 = dz^T a1 and
    dW1 = dz1^T agg, one reduction launch) equals two molclr_linear_wgrad_h3
    calls bit for bit, weights and biases, accumulating into non-zero grads."""
    from molclr_amd import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(rows)
    dz, a1 = torch.randn(rows, D, generator=g) * 1e-3, torch.randn(rows, 2 * D, generator=g)
    dz1, agg = torch.randn(rows, 2 * D, generator=g) * 1e-3, torch.randn(rows, D, generator=g)
    dz, a1, dz1, agg = (t.to(dev) for t in (dz, a1, dz1, agg))
    slots = torch.zeros(4, 2048, device=dev)
    for t, sl in zip((dz, a1, dz1, agg), slots):
        assert lib.molclr_absmax_f32(t.data_ptr(), t.shape[0], t.shape[1], t.shape[1],
                                     sl.data_ptr(), 0, ops._stream(t)) == 0
    init = [torch.randn(s, generator=g).to(dev) for s in ((D, 2 * D), (D,), (2 * D, D), (2 * D,))]
    one = [t.clone() for t in init]
    two = [t.clone() for t in init]
    st = ops._stream(dz)
    for (dy, sdy, x, sx, W, b) in ((dz, slots[0], a1, slots[1], one[0], one[1]),
                                   (dz1, slots[2], agg, slots[3], one[2], one[3])):
        wsb = lib.molclr_linear_wgrad_workspace_bytes(rows, dy.shape[1], x.shape[1])
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        assert lib.molclr_linear_wgrad_h3(dy.data_ptr(), sdy.data_ptr(), x.data_ptr(),
                                          sx.data_ptr(), W.data_ptr(), b.data_ptr(), rows,
                                          dy.shape[1], x.shape[1], dy.shape[1], x.shape[1], 1,
                                          ws.data_ptr(), wsb, st) == 0
    wsb = lib.molclr_linear_wgrad_h3_pair_workspace_bytes(rows, D, 2 * D, 2 * D, D)
    ws = torch.full((wsb + 1024,), 0x5A, dtype=torch.uint8, device=dev)
    assert lib.molclr_linear_wgrad_h3_pair(
        dz.data_ptr(), slots[0].data_ptr(), a1.data_ptr(), slots[1].data_ptr(), two[0].data_ptr(),
        two[1].data_ptr(), D, 2 * D, D, 2 * D, dz1.data_ptr(), slots[2].data_ptr(),
        agg.data_ptr(), slots[3].data_ptr(), two[2].data_ptr(), two[3].data_ptr(), 2 * D, D,
        2 * D, D, rows, 1, ws.data_ptr(), wsb, st) == 0, lib.molclr_last_error()
    torch.cuda.synchronize()
    assert bool((ws[wsb:] == 0x5A).all()), "wrote past the workspace"
    for a, b in zip(one, two):
        assert torch.equal(a, b)


def _wave_pairs(A):
    """The per-wave row-maximum pairs an aggregation producer writes
    (common.h row_max_waves): for every 64 consecutive float4 units of the
    row-major A, (max |.| of the wave's first row's units, of the next row's)."""
    M, K = A.shape
    d4 = K // 4
    u = A.abs().view(M * d4, 4).amax(1)
    nw = (M * d4 + 63) // 64
    out = torch.zeros(nw, 2, dtype=torch.float32)
    rows = torch.arange(M * d4) // d4
    for w in range(nw):
        lo, hi = 64 * w, min(64 * w + 64, M * d4)
        r0 = rows[lo].item()
        seg, rr = u[lo:hi], rows[lo:hi]
        out[w, 0] = seg[rr == r0].max()
        if (rr != r0).any():
            out[w, 1] = seg[rr != r0].max()
    return out


@pytest.mark.parametrize("M,N,K", [(30556, 600, 300), (1000, 400, 292), (70, 600, 300),
                                   (4099, 512, 300)])
@pytest.mark.parametrize("scales", ["tensor", "rows", "pairs"])
@pytest.mark.parametrize("epi,acc", [(0, 0), (1, 1), (2, 0), (3, 0)])
def test_gemm_h3_bs_matches_pp(dev, M, N, K, scales, epi, acc):
    """k_gemm_bs (the B-stationary h3 product of the K = 300 GIN products)
    against k_gemm_pp / k_gemm_q6 on the same inputs (molclr_gemm_f32_h3_impl
    1 vs 2): C, the ReLU bits, max |C|, max |A| and the row maxima bit for
    bit, for every epilogue, per-tensor / per-row / per-wave-pair A scales,
    accumulation, partial tiles and a row count leaving most blocks idle."""
    from molclr_amd import _lib
    if scales == "pairs" and (K // 4 < 64 or M * (K // 4) > 400_000):
        pytest.skip("pairs: a dense A of >= 64 float4s per row; host-built for small M")
    lib = _lib.load()
    g = torch.Generator().manual_seed(M + N + K + epi)
    A = torch.randn(M, K, generator=g) * torch.pow(10.0, -6 * torch.rand(M, 1, generator=g))
    W = (torch.rand(N, K, generator=g) * 2 - 1) / K ** 0.5
    bias = torch.randn(N, generator=g) * 0.1
    mask = torch.rand(M, N, generator=g) > 0.4
    words = (N + 31) // 32
    pos = torch.zeros(M, words * 32, dtype=torch.bool)
    pos[:, :N] = mask
    mb = ((pos.view(M, words, 32).long() << torch.arange(32)).sum(-1).remainder(1 << 32).t()
          .contiguous())
    mb = torch.where(mb >= (1 << 31), mb - (1 << 32), mb).to(torch.int32).to(dev)
    Ad, Wd, bd = A.to(dev), W.to(dev), bias.to(dev)
    planes = _h3_planes(lib, Wd, N, K, 0, dev)
    P = int(lib.molclr_gemm_row_parts(N))
    assert P == (N + 127) // 128
    if scales == "tensor":
        amax, parts = torch.zeros(2048, device=dev), 0
        assert lib.molclr_absmax_f32(Ad.data_ptr(), M, K, K, amax.data_ptr(), 0,
                                     ops._stream(Ad)) == 0
    elif scales == "rows":
        amax, parts = Ad.abs().amax(1).contiguous(), 1
    else:
        amax, parts = _wave_pairs(A).to(dev), -(K // 4)
    C0 = torch.randn(M, N, generator=g).to(dev)
    outs = []
    for impl in (1, 2):
        C = C0.clone()
        crow = torch.full((P, M), 7.0, device=dev)
        cmax = torch.zeros(2048, device=dev)
        aout = torch.zeros(2048, device=dev)
        bits = torch.zeros(words, M, dtype=torch.int32, device=dev)
        rc = lib.molclr_gemm_f32_h3_impl(
            Ad.data_ptr(), amax.data_ptr(), parts, planes.data_ptr(), C.data_ptr(), M, N, K, K, N,
            epi | (_lib.EPI_ACCUMULATE if acc else 0), bd.data_ptr(), None, 0,
            mb.data_ptr() if epi == 3 else None, cmax.data_ptr(), crow.data_ptr(),
            aout.data_ptr(), bits.data_ptr() if epi == 2 else None, ops._stream(Ad), impl)
        assert rc == 0, lib.molclr_last_error()
        torch.cuda.synchronize()
        outs.append((C, crow.amax(0), cmax.max(), aout.max(), bits))
    C, rmax, cmx, amx, bits = outs[1]
    # internal consistency of the bs outputs: row maxima, max |C|, max |A|, bits
    assert torch.equal(rmax, C.abs().amax(1))
    assert cmx.item() == C.abs().max().item() and amx.item() == Ad.abs().max().item()
    if epi == 2:
        pos = torch.zeros(M, words * 32, dtype=torch.bool, device=dev)
        pos[:, :N] = C > 0
        want = ((pos.view(M, words, 32).long() << torch.arange(32, device=dev)).sum(-1)
                .remainder(1 << 32).t())
        want = torch.where(want >= (1 << 31), want - (1 << 32), want).to(torch.int32)
        assert torch.equal(bits, want)
    if M >= 30556:
        # where the automatic choice is k_gemm_pp (one K group, >= 384 blocks),
        # k_gemm_bs is the same products in the same order: bit for bit
        for k, (a, b) in enumerate(zip(*outs)):
            assert torch.equal(a, b), k
    else:
        # q6 with two K groups sums in another order: both at fp32 accuracy
        ref = C0.double().cpu() * acc + A.double() @ W.double().t()
        if epi in (1, 2):
            ref = ref + bias.double()
        if epi == 2:
            ref = ref.clamp_min(0)
        if epi == 3:
            ref = ref * mask
        Cc = C.double().cpu()
        err = ((Cc - ref).norm(dim=1) / ref.norm(dim=1).clamp_min(1e-300))[ref.norm(dim=1) > 0]
        assert err.max().item() < 2e-6 if scales != "tensor" else rel(Cc, ref) < 2e-6


@pytest.mark.parametrize("M,N,K", [(30556, 600, 300), (1000, 400, 292), (70, 600, 300),
                                   (4099, 512, 300)])
@pytest.mark.parametrize("scales", ["tensor", "rows", "pairs"])
@pytest.mark.parametrize("epi,acc", [(0, 0), (1, 1), (2, 0), (3, 0)])
def test_gemm_h3_bs16(dev, M, N, K, scales, epi, acc):
    """k_gemm_bs16 (molclr_gemm_f32_h3_impl 3: the K = 300 products on the
    16 x 16 x 32 MFMA): C against fp64 at the h3 kernels' accuracy (row-wise
    2e-6), and its ReLU bits, row maxima, max |C| and max |A| consistent with
    its own C, for every epilogue and A-scale form, accumulation, partial
    tiles and mostly idle blocks."""
    from molclr_amd import _lib
    if scales == "pairs" and (K // 4 < 64 or M * (K // 4) > 400_000):
        pytest.skip("pairs: a dense A of >= 64 float4s per row; host-built for small M")
    lib = _lib.load()
    g = torch.Generator().manual_seed(M + N + K + epi + 1)
    A = torch.randn(M, K, generator=g) * torch.pow(10.0, -6 * torch.rand(M, 1, generator=g))
    W = (torch.rand(N, K, generator=g) * 2 - 1) / K ** 0.5
    bias = torch.randn(N, generator=g) * 0.1
    mask = torch.rand(M, N, generator=g) > 0.4
    words = (N + 31) // 32
    pos = torch.zeros(M, words * 32, dtype=torch.bool)
    pos[:, :N] = mask
    mb = ((pos.view(M, words, 32).long() << torch.arange(32)).sum(-1).remainder(1 << 32).t()
          .contiguous())
    mb = torch.where(mb >= (1 << 31), mb - (1 << 32), mb).to(torch.int32).to(dev)
    Ad, Wd, bd = A.to(dev), W.to(dev), bias.to(dev)
    planes = _h3_planes(lib, Wd, N, K, 0, dev)
    P = int(lib.molclr_gemm_row_parts(N))
    if scales == "tensor":
        amax, parts = torch.zeros(2048, device=dev), 0
        assert lib.molclr_absmax_f32(Ad.data_ptr(), M, K, K, amax.data_ptr(), 0,
                                     ops._stream(Ad)) == 0
    elif scales == "rows":
        amax, parts = Ad.abs().amax(1).contiguous(), 1
    else:
        amax, parts = _wave_pairs(A).to(dev), -(K // 4)
    C0 = torch.randn(M, N, generator=g).to(dev)
    C = C0.clone()
    crow = torch.full((P, M), 7.0, device=dev)
    cmax = torch.zeros(2048, device=dev)
    aout = torch.zeros(2048, device=dev)
    bits = torch.zeros(words, M, dtype=torch.int32, device=dev)
    rc = lib.molclr_gemm_f32_h3_impl(
        Ad.data_ptr(), amax.data_ptr(), parts, planes.data_ptr(), C.data_ptr(), M, N, K, K, N,
        epi | (_lib.EPI_ACCUMULATE if acc else 0), bd.data_ptr(), None, 0,
        mb.data_ptr() if epi == 3 else None, cmax.data_ptr(), crow.data_ptr(),
        aout.data_ptr(), bits.data_ptr() if epi == 2 else None, ops._stream(Ad), 3)
    assert rc == 0, lib.molclr_last_error()
    torch.cuda.synchronize()
    assert torch.equal(crow.amax(0), C.abs().amax(1))
    assert cmax.max().item() == C.abs().max().item()
    assert aout.max().item() == Ad.abs().max().item()
    if epi == 2:
        pos = torch.zeros(M, words * 32, dtype=torch.bool, device=dev)
        pos[:, :N] = C > 0
        want = ((pos.view(M, words, 32).long() << torch.arange(32, device=dev)).sum(-1)
                .remainder(1 << 32).t())
        want = torch.where(want >= (1 << 31), want - (1 << 32), want).to(torch.int32)
        assert torch.equal(bits, want)
    ref = C0.double().cpu() * acc + A.double() @ W.double().t()
    if epi in (1, 2):
        ref = ref + bias.double()
    if epi == 2:
        ref = ref.clamp_min(0)
    if epi == 3:
        ref = ref * mask
    Cc = C.double().cpu()
    err = ((Cc - ref).norm(dim=1) / ref.norm(dim=1).clamp_min(1e-300))[ref.norm(dim=1) > 0]
    assert err.max().item() < 2e-6 if scales != "tensor" else rel(Cc, ref) < 2e-6


@pytest.mark.parametrize("M,N,K", [(30556, 300, 600), (1000, 256, 580), (70, 300, 600),
                                   (4099, 320, 608)])
@pytest.mark.parametrize("scales", ["tensor", "rows"])
@pytest.mark.parametrize("epi,acc", [(0, 0), (1, 1), (2, 0), (3, 0)])
def test_gemm_h3_bs64(dev, M, N, K, scales, epi, acc):
    """The K = 600 products (lin2, dagg) on k_gemm_bsn with 64-column tiles
    (molclr_gemm_f32_h3_impl 3, 19 whole-K steps, an odd count): C against
    fp64 at the h3 kernels' accuracy, max |C| and max |A| consistent with it,
    every epilogue (ReLU mask from bits), accumulation, partial tiles."""
    from molclr_amd import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(M + N + K + epi + 2)
    A = torch.randn(M, K, generator=g) * torch.pow(10.0, -6 * torch.rand(M, 1, generator=g))
    W = (torch.rand(N, K, generator=g) * 2 - 1) / K ** 0.5
    bias = torch.randn(N, generator=g) * 0.1
    mask = torch.rand(M, N, generator=g) > 0.4
    words = (N + 31) // 32
    pos = torch.zeros(M, words * 32, dtype=torch.bool)
    pos[:, :N] = mask
    mb = ((pos.view(M, words, 32).long() << torch.arange(32)).sum(-1).remainder(1 << 32).t()
          .contiguous())
    mb = torch.where(mb >= (1 << 31), mb - (1 << 32), mb).to(torch.int32).to(dev)
    Ad, Wd, bd = A.to(dev), W.to(dev), bias.to(dev)
    planes = _h3_planes(lib, Wd, N, K, 0, dev)
    if scales == "tensor":
        amax, parts = torch.zeros(2048, device=dev), 0
        assert lib.molclr_absmax_f32(Ad.data_ptr(), M, K, K, amax.data_ptr(), 0,
                                     ops._stream(Ad)) == 0
    else:
        amax, parts = Ad.abs().amax(1).contiguous(), 1
    C0 = torch.randn(M, N, generator=g).to(dev)
    C = C0.clone()
    cmax = torch.zeros(2048, device=dev)
    aout = torch.zeros(2048, device=dev)
    rc = lib.molclr_gemm_f32_h3_impl(
        Ad.data_ptr(), amax.data_ptr(), parts, planes.data_ptr(), C.data_ptr(), M, N, K, K, N,
        epi | (_lib.EPI_ACCUMULATE if acc else 0), bd.data_ptr(), None, 0,
        mb.data_ptr() if epi == 3 else None, cmax.data_ptr(), None, aout.data_ptr(), None,
        ops._stream(Ad), 3)
    assert rc == 0, lib.molclr_last_error()
    torch.cuda.synchronize()
    assert cmax.max().item() == C.abs().max().item()
    assert aout.max().item() == Ad.abs().max().item()
    ref = C0.double().cpu() * acc + A.double() @ W.double().t()
    if epi in (1, 2):
        ref = ref + bias.double()
    if epi == 2:
        ref = ref.clamp_min(0)
    if epi == 3:
        ref = ref * mask
    Cc = C.double().cpu()
    err = ((Cc - ref).norm(dim=1) / ref.norm(dim=1).clamp_min(1e-300))[ref.norm(dim=1) > 0]
    assert err.max().item() < 2e-6 if scales != "tensor" else rel(Cc, ref) < 2e-6
