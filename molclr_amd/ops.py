"""Autograd functions over the C ABI (include/molclr.h).

Each function is one seam of the reference pre-training step, with an
explicit backward that calls the matching HIP kernel:

=====================  ==========================================================
function               reference (CameronDiao/MolCLR)
=====================  ==========================================================
``atom_embed``         models/ginet_molclr.py:103 (x_embedding1 + x_embedding2)
``gine_aggregate``     models/ginet_molclr.py:29-44 + PyG propagate(aggr='add')
``gin_mlp``            models/ginet_molclr.py:19-23,46-47 (GINEConv.update)
``linear``             nn.Linear (feat_lin, ginet_molclr.py:90)
``projection_head``    out_lin: Linear-ReLU-Linear (ginet_molclr.py:92-96)
``batch_norm``         ginet_molclr.py:107-111 (BatchNorm1d + ReLU + dropout 0)
``segment_pool``       ginet_molclr.py:113 (global_mean_pool / global_add_pool)
``gcn_conv``           models/gcn_molclr.py:62-88 (x @ W, propagate, + bias)
``l2_normalize``       molclr.py:63-64 (F.normalize)
``nt_xent``            utils/nt_xent.py:47-65 (NTXentLoss.forward)
=====================  ==========================================================

All tensors must be CUDA (HIP) fp32 and contiguous; there is no CPU path.
"""
from __future__ import annotations

import torch

import contextlib
import ctypes
import os
import functools
import weakref

from . import _lib
from ._lib import EPI_ACCUMULATE, EPI_BIAS, EPI_BIAS_RELU, EPI_NONE, EPI_RELU_MASK
from .data import DeviceGraph


@functools.lru_cache(maxsize=4096)
def _wsq(name: str, *args) -> int:
    """Cached workspace-size query (pure function of the sizes)."""
    return _lib.query(name, *args)


def _grad_sink(param, shape, device):
    """Where a parameter gradient is written.

    A parameter owned by FusedAdam (flag ``_molclr_fused_grad``) already has
    ``.grad`` as a view of the flat gradient buffer: the kernel adds into it
    directly (accumulate = 1) and the autograd function returns None for that
    input, so autograd launches no separate accumulation kernel.  Otherwise a
    fresh tensor is returned to autograd as usual.
    Returns (buffer, accumulate_flag, value_to_return)."""
    if param is not None and getattr(param, "_molclr_fused_grad", False) and param.grad is not None:
        return param.grad, 1, None
    t = torch.empty(shape, dtype=torch.float32, device=device)
    return t, 0, t


def _check(*ts):
    for t in ts:
        if t is None:
            continue
        if t.device.type != "cuda":
            raise RuntimeError("molclr_amd kernels run on the GPU only; got a %s tensor" % t.device)


_NULL_CTX = contextlib.nullcontext()


def _ws(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


def _c(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_contiguous() else t.contiguous()


def _stream(t: torch.Tensor) -> int:
    return _lib.stream_of(t.device)


class KernelTimer:
    """Per-kernel timing of the scatter-add and GEMM launches (used by bench.py).

    Durations come from the library's dispatch-recorded events
    (molclr_ktimer_*, hipExtLaunchKernelGGL): each sample is the kernel's own
    execution window, the same figure rocprofv3's kernel trace reports.  This
    class only counts calls and adds up their algorithmic work (bytes for the
    scatter-add, 2MNK flops for a GEMM, the similarity products' flops for
    NT-Xent: 2 n 2B C forward, twice that backward)."""

    KINDS = {"gine_aggregate_fwd": _lib.KTIMER_GINE_AGG, "gemm_f32": _lib.KTIMER_GEMM,
             "ntxent": _lib.KTIMER_NTXENT, "gcn_aggregate_fwd": _lib.KTIMER_GCN_AGG}

    def __init__(self, kinds=None):
        """``kinds``: the subset of KINDS to time (default all).  Every timed
        launch carries two dispatch events, so time only what is reported."""
        self.enabled = tuple(self.KINDS) if kinds is None else tuple(kinds)
        self.work = {k: 0.0 for k in self.KINDS}
        self.calls = {k: 0 for k in self.KINDS}
        mask = 0
        for k in self.enabled:
            mask |= self.KINDS[k]
        _lib.call("molclr_ktimer_start", mask)

    def add(self, kind, work):
        if kind not in self.enabled:
            return
        self.work[kind] += work
        self.calls[kind] += 1

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for kind, code in self.KINDS.items():
            ms = ctypes.c_double(0.0)
            n = ctypes.c_int64(0)
            _lib.call("molclr_ktimer_read", code, ctypes.addressof(ms), ctypes.addressof(n))
            if self.calls[kind]:
                out[kind] = {"launches": self.calls[kind], "kernel_launches": n.value,
                             "ms": ms.value, "work": self.work[kind]}
        _lib.call("molclr_ktimer_stop")
        return out


_TIMER: KernelTimer | None = None


def set_kernel_timer(timer: KernelTimer | None) -> None:
    global _TIMER
    _TIMER = timer


def _check_no_timer() -> None:
    """A HIP-graph capture cannot hold the timer's dispatch events."""
    if _TIMER is not None:
        raise RuntimeError("molclr_amd: stop the kernel timer before capturing a step")


# Gradient-ready hook of the data-parallel reducer
# (molclr_amd.distributed.OverlappedGradReducer): told when an encoder
# backward starts, given per-layer events the executor records, and told when
# the backward has been enqueued.
_GRAD_HOOK = None


def set_grad_hook(hook) -> None:
    global _GRAD_HOOK
    _GRAD_HOOK = hook


# Weight gradients of the readout heads on a second stream.  The heads'
# products (feat_lin, out_lin: 2B rows, ginet_molclr.py:90-96,114-115) are
# small GEMMs that leave most CUs idle, so with ``side=True`` (the models'
# _readout) a FusedAdam-owned weight's dW / db run on a side stream beside the
# data-gradient chain.  join_side() makes the current stream wait for them; the
# encoder backward (before the reducer's heads bucket), FusedAdam.step and the
# reducer's finish() call it.  Opt-in (MOLCLR_SIDE_WGRAD=1): bit-identical, but
# the captured c2 step measured slower with the fork than without (171.5k vs
# 176.0k molecules/s, two runs each on one box) -- the same finding as the
# encoder's per-layer second stream.
SIDE_WGRAD = os.environ.get("MOLCLR_SIDE_WGRAD", "0") == "1"
_SIDE_STREAMS = {}
_SIDE_PENDING = []


def _side_stream(dev) -> torch.cuda.Stream:
    s = _SIDE_STREAMS.get(dev.index)
    if s is None:
        s = _SIDE_STREAMS[dev.index] = torch.cuda.Stream(dev)
    return s


def join_side() -> None:
    """The current stream waits for every pending side-stream weight gradient."""
    while _SIDE_PENDING:
        dev, ev = _SIDE_PENDING.pop()
        torch.cuda.current_stream(dev).wait_event(ev)


def _grad_events(grads_struct, L, owned):
    """Start the hook's heads bucket and fill the executor's done-events."""
    join_side()  # the heads' gradients are final before their bucket starts
    hook = _GRAD_HOOK
    if hook is None or not owned:
        return None
    hook.encoder_backward_begin()
    ev = hook.layer_event_handles()
    if ev is not None:
        for l in range(L):
            grads_struct.layer_done[l] = ev[l]
        grads_struct.embed_done = ev[L]
    return hook


# ---------------------------------------------------------------------------
# GEMM helpers
# ---------------------------------------------------------------------------
def gemm(A, B, M, N, K, lda, ldb, a_kmajor, b_kmajor, epi=EPI_NONE, bias=None, aux=None,
         out=None, accumulate=0, impl=-1):
    """C[M,N] = op(A) op(B) (+ epilogue, + C if accumulate), see molclr_gemm_f32
    (``impl``: molclr_gemm_f32_impl's choice, -1 = automatic)."""
    dev = A.device
    if out is None:
        out = torch.empty(M, N, dtype=torch.float32, device=dev)
    if accumulate:
        epi |= EPI_ACCUMULATE
    ws_bytes = _wsq("molclr_gemm_f32_workspace_bytes", M, N, K)
    ws = _ws(ws_bytes, dev) if ws_bytes else None
    _lib.call("molclr_gemm_f32_impl", A.data_ptr(), B.data_ptr(), out.data_ptr(), M, N, K, lda,
              ldb, out.stride(0), int(a_kmajor), int(b_kmajor), epi, _lib.ptr(bias), _lib.ptr(aux),
              aux.stride(0) if aux is not None else 0, _lib.ptr(ws), ws_bytes, _stream(A),
              int(impl))
    if _TIMER is not None:
        _TIMER.add("gemm_f32", 2.0 * M * N * K)
    return out


# Pre-split weight planes (molclr_bplanes_make), cached per weight tensor and
# invalidated when the tensor changes: torch's version counter covers in-place
# torch ops (load_state_dict, torch.optim), PARAM_GENERATION covers FusedAdam,
# whose kernel writes the parameters through raw pointers.
USE_BPLANES = True
PARAM_GENERATION = [0]
_PLANES: dict = {}


def bump_param_generation() -> None:
    PARAM_GENERATION[0] += 1


_PLANE_FNS = {"x6": ("molclr_bplanes_bytes", "molclr_bplanes_make_batch"),
              "h3": ("molclr_hplanes_bytes", "molclr_hplanes_make_batch")}


def weight_planes(W, N, K, ldb, b_kmajor, kind: str = "x6") -> torch.Tensor:
    """B(k, n) stored in W (molclr_gemm_f32's B layout) as a GEMM operand image:
    kind "x6" = split-bf16 planes (molclr_bplanes_make), "h3" = fp16 two-part
    planes and their max slot (molclr_hplanes_make_batch).

    After an optimizer step every cached image is stale: the first lookup
    regenerates all live ones in one batched launch per kind, not one launch
    per weight and orientation."""
    key = (W.data_ptr(), N, K, ldb, int(b_kmajor), kind)
    gen = PARAM_GENERATION[0]
    ent = _PLANES.get(key)
    if ent is not None and ent[1]() is W:
        if ent[0] == (W._version, gen):
            return _keep_image(ent[3])
        if ent[0][1] != gen:
            _refresh_planes(gen)
            ent = _PLANES[key]
        if ent[0] != (W._version, gen):
            # changed in place within the generation: regenerate into the SAME
            # image -- a captured step writes (and its replays read) this
            # address, so it must never be freed while W lives
            _make_planes(kind, [(W, ent[2], ent[3])])
            ent = _PLANES[key] = ((W._version, gen), ent[1], ent[2], ent[3])
        return _keep_image(ent[3])
    # drop entries of dead tensors on every insert: a padded weight (emb_dim
    # not a multiple of the kernels' width) is a new tensor each call, and its
    # planes must not stay pinned in HBM
    for k in [k for k, e in _PLANES.items() if e[1]() is None]:
        _drop_image(_PLANES.pop(k)[3])
    nbytes = _wsq(_PLANE_FNS[kind][0], N, K)
    planes = _new_image(nbytes, W.device)
    _make_planes(kind, [(W, (N, K, ldb, int(b_kmajor)), planes)])
    _PLANES[key] = ((W._version, gen), weakref.ref(W), (N, K, ldb, int(b_kmajor)), planes)
    return _keep_image(planes)


# Weight images are state that outlives a step: they must not come from a
# graph's private memory pool.  CapturedTrainStep runs the step once as a dry
# run (_lib.dry_run: every library call skipped) before capturing it, so every
# image the step uses already exists when the capture starts and the capture
# only records its regeneration.  The capture also keeps a reference to every
# image its graph writes (CAPTURE_KEEP, held by the captured entry), so an
# image a live graph regenerates can never be freed and handed to someone else.
CAPTURE_KEEP: list | None = None


def _new_image(nbytes: int, device) -> torch.Tensor:
    return torch.empty(nbytes // 2, dtype=torch.int16, device=device)


def _keep_image(planes: torch.Tensor) -> torch.Tensor:
    if CAPTURE_KEEP is not None:
        CAPTURE_KEEP.append(planes)
    return planes


def _drop_image(planes: torch.Tensor) -> None:
    """An image of a dead weight leaves the cache (the caching allocator
    reuses it in stream order)."""
    del planes


def _make_planes(kind, jobs) -> None:
    n = len(jobs)
    arr = lambda vals, ct: (ct * n)(*vals)  # noqa: E731
    _lib.call(_PLANE_FNS[kind][1], n,
              arr([j[0].data_ptr() for j in jobs], ctypes.c_void_p),
              arr([j[1][0] for j in jobs], ctypes.c_int64),
              arr([j[1][1] for j in jobs], ctypes.c_int64),
              arr([j[1][2] for j in jobs], ctypes.c_int64),
              arr([j[1][3] for j in jobs], ctypes.c_int),
              arr([j[2].data_ptr() for j in jobs], ctypes.c_void_p), _stream(jobs[0][2]))


# While a step is being captured (molclr_amd.graph_step): the ids of its
# model's parameters.  The capture then regenerates only THEIR images: an image
# of another model refreshed inside the graph would be written by every replay
# even after that model's image was freed and its memory reused.
CAPTURE_SCOPE: set | None = None


def _refresh_planes(gen: int) -> None:
    """Regenerate every live cached image of an older generation, batched
    (while capturing: the captured model's only)."""
    jobs = {}
    scope = CAPTURE_SCOPE
    for k, (tok, ref, shape, planes) in list(_PLANES.items()):
        W = ref()
        if W is None:
            _drop_image(_PLANES.pop(k)[3])
            continue
        if scope is not None and id(W) not in scope:
            continue
        if tok[1] != gen and W.data_ptr() == k[0]:
            jobs.setdefault(k[5], []).append((k, W, shape, planes))
    for kind, js in jobs.items():
        _make_planes(kind, [(W, shape, planes) for _, W, shape, planes in js])
        for k, W, shape, planes in js:
            _PLANES[k] = ((W._version, gen), weakref.ref(W), shape, _keep_image(planes))


# fp32 GEMMs of the GIN MLP backward (data and weight gradients): "h3" = three
# fp16 MFMAs per product with power-of-two scaling (molclr_gemm_f32_h3 with
# row-wise scales, molclr_linear_wgrad_h3), "x6" = six split-bf16 MFMAs.
# H3_FORWARD puts the forward products on h3 too, A scaled row by row (the
# default: elementwise as accurate as the reference's fp32 sgemm, no more
# ReLU decisions flipped against fp64 -- tools/h3_forward_flips.py;
# MOLCLR_H3_FORWARD=0 keeps them on x6).  The encoder executor reads the same
# switches, so both paths issue identical kernels.
FP32_GEMM = os.environ.get("MOLCLR_FP32_GEMM", "h3")
H3_FORWARD = os.environ.get("MOLCLR_H3_FORWARD", "1") == "1"


MAX_SLOT = 64 * 32  # floats per max |x| slot (molclr_absmax_f32: 64 entries, 128 B apart)


def absmax(x, out=None, accumulate=0) -> torch.Tensor:
    """max |x| of a row-major fp32 matrix into a device max slot (MAX_SLOT
    floats whose max is the value)."""
    if out is None:
        out = torch.empty(MAX_SLOT, dtype=torch.float32, device=x.device)
    rows, cols = x.shape
    _lib.call("molclr_absmax_f32", x.data_ptr(), rows, cols, x.stride(0), out.data_ptr(),
              int(accumulate), _stream(x))
    return out


def row_parts(N: int) -> int:
    """Partial row-max arrays a GEMM with N output columns writes (crow)."""
    return int(_lib.load().molclr_gemm_row_parts(N))


def gemm_h3(A, amax, W, N, K, ldb, b_kmajor, epi=EPI_NONE, bias=None, aux=None, cmax=None,
            rowwise=0, crow=None, amax_out=None, mask_bits=None, bits_out=None):
    """C = epilogue(A B) with B(k, n) in W, by molclr_gemm_f32_h3_bits.  amax:
    A's max slot, or (rowwise = P > 0) its row maxima as P partial arrays [P][M];
    cmax (zeroed) receives max |C|, crow [row_parts(N)][M] C's row maxima,
    bits_out (BIAS_RELU) C's ReLU mask as bits."""
    _check(A, W)
    M = A.shape[0]
    planes = weight_planes(W, N, K, ldb, b_kmajor, "h3")
    out = torch.empty(M, N, dtype=torch.float32, device=A.device)
    _lib.call("molclr_gemm_f32_h3_bits", A.data_ptr(), amax.data_ptr(), int(rowwise),
              planes.data_ptr(),
              out.data_ptr(), M, N, K, A.stride(0), out.stride(0), epi, _lib.ptr(bias),
              _lib.ptr(aux), aux.stride(0) if aux is not None else 0, _lib.ptr(mask_bits),
              _lib.ptr(cmax), _lib.ptr(crow), _lib.ptr(amax_out), _lib.ptr(bits_out), _stream(A))
    if _TIMER is not None:
        _TIMER.add("gemm_f32", 2.0 * M * N * K)
    return out


def linear_wgrad_h3(dy, dymax, x, xmax, W_param, b_param):
    """dW = dy^T x and db = Σ dy by molclr_linear_wgrad_h3 (into the FusedAdam
    .grad when it owns them).  Returns (dW, db) as linear_bwd does."""
    M, K = x.shape
    N = dy.shape[1]
    wbuf, wacc, dW = _grad_sink(W_param, (N, K), dy.device)
    bbuf, bacc, db = _grad_sink(b_param, (N,), dy.device)
    if wacc != bacc:
        wbuf, wacc, dW = _grad_sink(None, (N, K), dy.device)
        bbuf, bacc, db = _grad_sink(None, (N,), dy.device)
    ws_bytes = _wsq("molclr_linear_wgrad_workspace_bytes", M, N, K)
    ws = _ws(ws_bytes, dy.device)
    _lib.call("molclr_linear_wgrad_h3", dy.data_ptr(), dymax.data_ptr(), x.data_ptr(),
              xmax.data_ptr(), wbuf.data_ptr(), bbuf.data_ptr(), M, N, K, dy.stride(0),
              x.stride(0), wacc, ws.data_ptr(), ws_bytes, _stream(dy))
    if _TIMER is not None:
        _TIMER.add("gemm_f32", 2.0 * M * N * K)
    return dW, db


def gcn_h3_ok(rows, D) -> bool:
    """Shapes GCNConv's h3 backward takes (else x6)."""
    return FP32_GEMM == "h3" and D % 4 == 0 and D <= 1024 and rows > 0


def h3_ok(rows, D) -> bool:
    """Shapes the h3 GIN-MLP GEMMs take (else the x6 kernels run)."""
    return FP32_GEMM == "h3" and D % 4 == 0 and 2 * D <= 1024 and rows > 0


def gemm_w(A, W, M, N, K, lda, ldb, a_kmajor, b_kmajor, epi=EPI_NONE, bias=None, aux=None,
           out=None, accumulate=0, tile=0):
    """gemm() whose B operand is a weight: through its cached pre-split planes
    (molclr_gemm_f32_bplanes; ``tile``: molclr_gemm_f32_bplanes_tile's choice)."""
    if not USE_BPLANES:
        return gemm(A, W, M, N, K, lda, ldb, a_kmajor, b_kmajor, epi, bias, aux, out, accumulate)
    _check(A, W)
    planes = weight_planes(W, N, K, ldb, b_kmajor)
    dev = A.device
    if out is None:
        out = torch.empty(M, N, dtype=torch.float32, device=dev)
    if accumulate:
        epi |= EPI_ACCUMULATE
    ws_bytes = _wsq("molclr_gemm_f32_workspace_bytes", M, N, K)
    ws = _ws(ws_bytes, dev) if ws_bytes else None
    _lib.call("molclr_gemm_f32_bplanes_tile", A.data_ptr(), planes.data_ptr(), out.data_ptr(), M,
              N, K, lda, out.stride(0), int(a_kmajor), epi, _lib.ptr(bias), _lib.ptr(aux),
              aux.stride(0) if aux is not None else 0, _lib.ptr(ws), ws_bytes, _stream(A),
              int(tile))
    if _TIMER is not None:
        _TIMER.add("gemm_f32", 2.0 * M * N * K)
    return out


def linear_fwd(x, W, b, relu=False):
    """y = x W^T + b (nn.Linear), optional fused ReLU."""
    M, K = x.shape
    N = W.shape[0]
    epi = EPI_BIAS_RELU if relu else EPI_BIAS
    return gemm_w(x, W, M, N, K, K, K, False, False, epi, bias=b)


def colsum(x, out=None, accumulate=0):
    rows, cols = x.shape
    ws_bytes = _wsq("molclr_colsum_f32_workspace_bytes", rows, cols)
    ws = _ws(ws_bytes, x.device)
    if out is None:
        out = torch.empty(cols, dtype=torch.float32, device=x.device)
    _lib.call("molclr_colsum_f32", x.data_ptr(), out.data_ptr(), rows, cols, x.stride(0),
              int(accumulate), ws.data_ptr(), ws_bytes, _stream(x))
    return out


def linear_bwd(dy, x, W, need_x=True, need_w=True, need_b=True, relu_mask_src=None,
               W_param=None, b_param=None, side=False):
    """Backward of y = x W^T + b.  Returns (dx, dW, db); dW / db are None when
    they were accumulated straight into a FusedAdam-owned .grad (``side``: on
    the side stream then, see join_side)."""
    M, K = x.shape
    N = W.shape[0]
    dx = dW = db = None
    if need_w and need_b:
        # dW[N,K] = dy^T x and db = Σ_rows dy in one pass (molclr_linear_wgrad)
        wbuf, wacc, dW = _grad_sink(W_param, (N, K), dy.device)
        bbuf, bacc, db = _grad_sink(b_param, (N,), dy.device)
        if wacc != bacc:  # mixed ownership: fresh buffers for both
            wbuf, wacc, dW = _grad_sink(None, (N, K), dy.device)
            bbuf, bacc, db = _grad_sink(None, (N,), dy.device)
        side = side and SIDE_WGRAD and wacc == 1 and _TIMER is None
        ss = _side_stream(dy.device) if side else None
        if side:
            ss.wait_stream(torch.cuda.current_stream(dy.device))
        with torch.cuda.stream(ss) if side else _NULL_CTX:
            ws_bytes = _wsq("molclr_linear_wgrad_workspace_bytes", M, N, K)
            ws = _ws(ws_bytes, dy.device)  # allocated on (and freed to) the side stream
            _lib.call("molclr_linear_wgrad", dy.data_ptr(), x.data_ptr(), wbuf.data_ptr(),
                      bbuf.data_ptr(), M, N, K, dy.stride(0), x.stride(0), wacc, ws.data_ptr(),
                      ws_bytes, _stream(dy))
        if side:
            dy.record_stream(ss)
            x.record_stream(ss)
            ev = torch.cuda.Event()
            ev.record(ss)
            _SIDE_PENDING.append((dy.device, ev))
        if _TIMER is not None:
            _TIMER.add("gemm_f32", 2.0 * M * N * K)
    elif need_w:
        # dW[N,K] = dy^T x : A = dy (K-major, lda=N), B = x (K-major, ldb=K)
        buf, acc, dW = _grad_sink(W_param, (N, K), dy.device)
        gemm(dy, x, N, K, M, N, K, True, True, out=buf, accumulate=acc)
    elif need_b:
        buf, acc, db = _grad_sink(b_param, (N,), dy.device)
        colsum(dy, out=buf, accumulate=acc)
    if need_x:
        # dx[M,K] = dy W : B(k=n, j) = W[n, j] (K-major, ldb=K)
        epi = EPI_RELU_MASK if relu_mask_src is not None else EPI_NONE
        dx = gemm_w(dy, W, M, K, N, N, K, False, True, epi, aux=relu_mask_src)
    return dx, dW, db


def gine_aggregate_bytes(N: int, D: int, E: int, elem_bytes: int = 4) -> int:
    """Compulsory HBM bytes of one molclr_gine_aggregate_fwd launch: read x and
    write the output once (2*N*D*s, s = 4 fp32 / 2 bf16) and the 16-byte
    neighbour slots of every node (16N); the 15 x D combined edge table is
    cache-resident, and the CSR tail of the few rows of degree > 4 is not
    counted.  (E is kept for the signature: the slot layout makes the
    compulsory bytes independent of it.)"""
    return 2 * N * D * elem_bytes + 16 * N


def edge_tables_combine(E1s, E2s) -> torch.Tensor:
    """Ec[l] = E1_l[bt] + E2_l[bd] for every (bt, bd), all layers in one launch
    ([L, 15, D]); not differentiable (gradients flow through the aggregation's
    count-weighted backward to E1/E2)."""
    L = len(E1s)
    if L == 0 or L > _lib.MAX_LAYERS:
        raise ValueError(f"edge_tables_combine: {L} layers (1..{_lib.MAX_LAYERS})")
    _check(*E1s, *E2s)
    E1s = [_c(e.detach()) for e in E1s]
    E2s = [_c(e.detach()) for e in E2s]
    D = E1s[0].shape[1]
    Ec = torch.empty(L, _lib.NUM_ECOMB, D, dtype=torch.float32, device=E1s[0].device)
    arr1 = (ctypes.c_void_p * L)(*[e.data_ptr() for e in E1s])
    arr2 = (ctypes.c_void_p * L)(*[e.data_ptr() for e in E2s])
    _lib.call("molclr_edge_tables_combine", L, arr1, arr2, Ec.data_ptr(), D, _stream(Ec))
    return Ec


# ---------------------------------------------------------------------------
# autograd functions
# ---------------------------------------------------------------------------
class _AtomEmbed(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_idx, X1, X2, status=None):
        _check(x_idx, X1, X2)
        x_idx = _c(x_idx.to(torch.long))
        N = x_idx.shape[0]
        D = X1.shape[1]
        h = torch.empty(N, D, dtype=torch.float32, device=X1.device)
        _lib.call("molclr_atom_embed_fwd", x_idx.data_ptr(), X1.data_ptr(), X2.data_ptr(),
                  h.data_ptr(), N, D, X1.shape[0], X2.shape[0], _lib.ptr(status), _stream(X1))
        ctx.save_for_backward(x_idx)
        ctx.shapes = (X1.shape[0], X2.shape[0], D)
        ctx.params = (X1, X2)
        return h

    @staticmethod
    def backward(ctx, dh):
        (x_idx,) = ctx.saved_tensors
        n1, n2, D = ctx.shapes
        dh = _c(dh)
        N = x_idx.shape[0]
        X1, X2 = ctx.params
        b1, acc1, r1 = _grad_sink(X1, (n1, D), dh.device)
        b2, acc2, r2 = _grad_sink(X2, (n2, D), dh.device)
        if acc1 != acc2:  # mixed ownership: write fresh tensors for both
            b1, acc1, r1 = _grad_sink(None, (n1, D), dh.device)
            b2, acc2, r2 = _grad_sink(None, (n2, D), dh.device)
        ws_bytes = _wsq("molclr_atom_embed_bwd_workspace_bytes", N, D, n1, n2)
        ws = _ws(ws_bytes, dh.device)
        _lib.call("molclr_atom_embed_bwd", x_idx.data_ptr(), dh.data_ptr(), b1.data_ptr(),
                  b2.data_ptr(), N, D, n1, n2, acc1, ws.data_ptr(), ws_bytes, _stream(dh))
        return None, r1, r2, None


class _GINEAggregate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, E1, E2, graph: DeviceGraph, Ec):
        _check(h, E1, E2, Ec)
        h = _c(h)
        N, D = h.shape
        if Ec is None:
            Ec = edge_tables_combine([E1], [E2])[0]
        if Ec.shape != (_lib.NUM_ECOMB, D) or not Ec.is_contiguous():
            raise ValueError(f"gine_aggregate: Ec must be a contiguous [15, {D}] table")
        out = torch.empty_like(h)
        _lib.call("molclr_gine_aggregate_fwd", h.data_ptr(), graph.rowptr.data_ptr(),
                  graph.col.data_ptr(), graph.ecode.data_ptr(), graph.nbr.data_ptr(),
                  Ec.data_ptr(), out.data_ptr(), N, D, _stream(h))
        if _TIMER is not None:
            _TIMER.add("gine_aggregate_fwd", gine_aggregate_bytes(N, D, graph.num_edges))
        ctx.graph = graph
        ctx.shapes = (N, D, E1.shape[0], E2.shape[0])
        ctx.params = (E1, E2)
        return out

    @staticmethod
    def backward(ctx, g):
        g = _c(g)
        N, D, n1, n2 = ctx.shapes
        graph = ctx.graph
        need_x, need_e1, need_e2 = ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        dx = torch.empty_like(g) if need_x else None
        E1, E2 = ctx.params
        b1 = b2 = r1 = r2 = None
        acc = 0
        if need_e1 and need_e2:
            b1, a1, r1 = _grad_sink(E1, (n1, D), g.device)
            b2, a2, r2 = _grad_sink(E2, (n2, D), g.device)
            if a1 != a2:
                b1, a1, r1 = _grad_sink(None, (n1, D), g.device)
                b2, a2, r2 = _grad_sink(None, (n2, D), g.device)
            acc = a1
        elif need_e1 or need_e2:
            if need_e1:
                b1, _, r1 = _grad_sink(None, (n1, D), g.device)
            else:
                b2, _, r2 = _grad_sink(None, (n2, D), g.device)
        ws_bytes = _wsq("molclr_gine_aggregate_bwd_workspace_bytes", N, D)
        ws = _ws(ws_bytes, g.device)
        _lib.call("molclr_gine_aggregate_bwd", g.data_ptr(), graph.rowptr_t.data_ptr(),
                  graph.col_t.data_ptr(), graph.nbr_t.data_ptr(), graph.ecount.data_ptr(),
                  _lib.ptr(dx), _lib.ptr(b1), _lib.ptr(b2), N, D, acc, ws.data_ptr(), ws_bytes,
                  _stream(g))
        return dx, r1, r2, None, None


class _MLP(torch.autograd.Function):
    """Linear -> ReLU -> Linear with the ReLU fused into the first GEMM's
    epilogue (forward) and into the dZ1 GEMM's epilogue (backward)."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2, side=False):
        _check(x, W1, b1, W2, b2)
        x = _c(x)
        ctx.side = side
        M, D = x.shape
        ctx.h3 = h3_ok(M, D) and W1.shape == (2 * D, D) and W2.shape == (D, 2 * D)
        if ctx.h3:
            # the executor's order: max |x| and its row maxima by a pass, then
            # the products (row-wise h3 when H3_FORWARD, else x6 with max |a1| by
            # a pass); the max slots serve the h3 weight gradients
            slots = torch.zeros(2, MAX_SLOT, dtype=torch.float32, device=x.device)
            # a1's ReLU mask as bits for the dz1 product, from the first product
            ctx.bits = torch.empty((2 * D + 31) // 32, M, dtype=torch.int32, device=x.device)
            if H3_FORWARD:
                P = row_parts(2 * D)
                rx = torch.empty(M, dtype=torch.float32, device=x.device)
                ra1 = torch.empty(P, M, dtype=torch.float32, device=x.device)
                _lib.call("molclr_absmax_rows_f32", x.data_ptr(), M, D, x.stride(0),
                          rx.data_ptr(), slots[0].data_ptr(), 1, _stream(x))
                a1 = gemm_h3(x, rx, W1, 2 * D, D, D, 0, EPI_BIAS_RELU, bias=b1,
                             cmax=slots[1], rowwise=1, crow=ra1, bits_out=ctx.bits)
                z = gemm_h3(a1, ra1, W2, D, 2 * D, 2 * D, 0, EPI_BIAS, bias=b2, rowwise=P)
            else:
                # the first product (q6, x6 planes) also yields max |x| and max |a1|
                a1 = torch.empty(M, 2 * D, dtype=torch.float32, device=x.device)
                ws_bytes = _wsq("molclr_gemm_f32_workspace_bytes", M, 2 * D, D)
                ws = _ws(ws_bytes, x.device) if ws_bytes else None
                _lib.call("molclr_gemm_f32_bplanes_max", x.data_ptr(),
                          weight_planes(W1, 2 * D, D, D, 0).data_ptr(), a1.data_ptr(), M, 2 * D,
                          D, x.stride(0), a1.stride(0), EPI_BIAS_RELU, b1.data_ptr(), None, 0,
                          slots[0].data_ptr(), slots[1].data_ptr(), None, ctx.bits.data_ptr(),
                          _lib.ptr(ws), ws_bytes, _stream(x))
                if _TIMER is not None:
                    _TIMER.add("gemm_f32", 2.0 * M * 2 * D * D)
                z = linear_fwd(a1, W2, b2, relu=False)
            ctx.slots = slots
        else:
            a1 = linear_fwd(x, W1, b1, relu=True)
            z = linear_fwd(a1, W2, b2, relu=False)
        ctx.save_for_backward(x, W1, W2, a1)
        ctx.params = (W1, b1, W2, b2)
        return z

    @staticmethod
    def backward(ctx, dz):
        x, W1, W2, a1 = ctx.saved_tensors
        pW1, pb1, pW2, pb2 = ctx.params
        dz = _c(dz)
        need = ctx.needs_input_grad
        if ctx.h3 and all(need[1:5]):
            # the executor's h3 order: dz1 (relu mask of a1; max |dz1| and its row
            # maxima from its epilogue), dW2 (+db2), dW1 (+db1), dx
            D = x.shape[1]
            slots = ctx.slots
            M = x.shape[0]
            P = row_parts(2 * D)
            bslots = torch.zeros(2, MAX_SLOT, dtype=torch.float32, device=dz.device)
            rdz = torch.empty(M, dtype=torch.float32, device=dz.device)      # row maxima of dz
            rdz1 = torch.empty(P, M, dtype=torch.float32, device=dz.device)  # ... of dz1
            _lib.call("molclr_absmax_rows_f32", dz.data_ptr(), M, D, dz.stride(0),
                      rdz.data_ptr(), bslots[0].data_ptr(), 1, _stream(dz))
            dz1 = gemm_h3(dz, rdz, W2, 2 * D, D, 2 * D, 1, EPI_RELU_MASK, aux=a1,
                          cmax=bslots[1], rowwise=1, crow=rdz1, mask_bits=ctx.bits)
            dW2, db2 = linear_wgrad_h3(dz, bslots[0], a1, slots[1], pW2, pb2)
            dW1, db1 = linear_wgrad_h3(dz1, bslots[1], x, slots[0], pW1, pb1)
            dx = (gemm_h3(dz1, rdz1, W1, D, 2 * D, D, 1, rowwise=P) if need[0] else None)
            return dx, dW1, db1, dW2, db2, None
        # through the second Linear; ReLU mask of a1 fused into dz1's epilogue
        dz1, dW2, db2 = linear_bwd(dz, a1, W2, need_x=True, need_w=need[3], need_b=need[4],
                                   relu_mask_src=a1, W_param=pW2, b_param=pb2, side=ctx.side)
        dx, dW1, db1 = linear_bwd(dz1, x, W1, need_x=need[0], need_w=need[1], need_b=need[2],
                                  W_param=pW1, b_param=pb1, side=ctx.side)
        return dx, dW1, db1, dW2, db2, None


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, b, side=False):
        _check(x, W, b)
        x = _c(x)
        ctx.save_for_backward(x, W)
        ctx.params = (W, b)
        ctx.side = side
        return linear_fwd(x, W, b)

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        need = ctx.needs_input_grad
        dx, dW, db = linear_bwd(_c(dy), x, W, need[0], need[1], need[2],
                                W_param=ctx.params[0], b_param=ctx.params[1], side=ctx.side)
        return dx, dW, db, None


class _BatchNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, gamma, beta, running_mean, running_var, training, momentum, eps, relu,
                num_batches_tracked=None):
        _check(z, gamma, beta)
        z = _c(z)
        N, D = z.shape
        y = torch.empty_like(z)
        save_mean = torch.empty(D, dtype=torch.float32, device=z.device)
        save_invstd = torch.empty(D, dtype=torch.float32, device=z.device)
        ws_bytes = _wsq("molclr_batchnorm_workspace_bytes", N, D)
        ws = _ws(ws_bytes, z.device)
        _lib.call("molclr_batchnorm_fwd", z.data_ptr(), _lib.ptr(gamma), _lib.ptr(beta),
                  _lib.ptr(running_mean), _lib.ptr(running_var), _lib.ptr(num_batches_tracked),
                  y.data_ptr(),
                  save_mean.data_ptr(), save_invstd.data_ptr(), N, D, float(momentum),
                  float(eps), int(bool(training)), int(bool(relu)), ws.data_ptr(), ws_bytes,
                  _stream(z))
        ctx.save_for_backward(z, gamma, beta, save_mean, save_invstd)
        ctx.params = (gamma, beta)
        ctx.relu = bool(relu)
        ctx.training = bool(training)
        return y

    @staticmethod
    def backward(ctx, dy):
        if not ctx.training:
            raise NotImplementedError(
                "molclr_amd: backward through eval-mode BatchNorm is not supported "
                "(the reference only evaluates under torch.no_grad, molclr.py:162)")
        z, gamma, beta, save_mean, save_invstd = ctx.saved_tensors
        dy = _c(dy)
        N, D = z.shape
        dz = torch.empty_like(z)
        pg, pb = ctx.params
        bg, ag, rg = _grad_sink(pg, (D,), z.device)
        bb, ab, rb = _grad_sink(pb, (D,), z.device)
        if ag != ab:
            bg, ag, rg = _grad_sink(None, (D,), z.device)
            bb, ab, rb = _grad_sink(None, (D,), z.device)
        ws_bytes = _wsq("molclr_batchnorm_workspace_bytes", N, D)
        ws = _ws(ws_bytes, z.device)
        _lib.call("molclr_batchnorm_bwd", dy.data_ptr(), z.data_ptr(), _lib.ptr(gamma),
                  _lib.ptr(beta), save_mean.data_ptr(), save_invstd.data_ptr(), dz.data_ptr(),
                  bg.data_ptr(), bb.data_ptr(), N, D, int(ctx.relu), ag, ws.data_ptr(),
                  ws_bytes, _stream(z))
        return dz, rg, rb, None, None, None, None, None, None, None


POOL_MODES = {"mean": 0, "add": 1}


class _SegmentPool(torch.autograd.Function):
    """Pooling over graph_ptr; bf16 node embeddings pool into fp32 (the
    projection heads stay fp32) and receive a bf16 gradient."""

    @staticmethod
    def forward(ctx, h, graph: DeviceGraph, mode: int):
        _check(h)
        h = _c(h)
        N, D = h.shape
        G = graph.num_graphs
        out = torch.empty(G, D, dtype=torch.float32, device=h.device)
        bf = h.dtype == torch.bfloat16
        if not bf and h.dtype != torch.float32:
            raise TypeError(f"segment_pool: {h.dtype} node embeddings (fp32 / bf16)")
        _lib.call("molclr_segment_pool_fwd_bf16" if bf else "molclr_segment_pool_fwd", h.data_ptr(),
                  graph.graph_ptr.data_ptr(), out.data_ptr(), G, D, mode, _stream(h))
        ctx.graph, ctx.mode, ctx.N, ctx.dtype = graph, mode, N, h.dtype
        return out

    @staticmethod
    def backward(ctx, dout):
        dout = _c(dout.to(torch.float32))
        G, D = dout.shape
        dh = torch.empty(ctx.N, D, dtype=ctx.dtype, device=dout.device)
        bf = ctx.dtype == torch.bfloat16
        _lib.call("molclr_segment_pool_bwd_bf16" if bf else "molclr_segment_pool_bwd",
                  dout.data_ptr(), ctx.graph.graph_ptr.data_ptr(), dh.data_ptr(), ctx.N, G, D,
                  ctx.mode, _stream(dout))
        return dh, None, None


class _SegmentMax(torch.autograd.Function):
    """global_max_pool (PyG 1.6.3 -> torch_scatter 2.0.6 scatter_max): the
    gradient goes to the arg-max node of each (graph, column)."""

    @staticmethod
    def forward(ctx, h, graph: DeviceGraph):
        _check(h)
        h = _c(h)
        N, D = h.shape
        G = graph.num_graphs
        if h.dtype not in (torch.float32, torch.bfloat16):
            raise TypeError(f"segment_max: {h.dtype} node embeddings (fp32 / bf16)")
        dt = _lib.DTYPE_BF16 if h.dtype == torch.bfloat16 else _lib.DTYPE_F32
        out = torch.empty(G, D, dtype=torch.float32, device=h.device)
        arg = torch.empty(G, D, dtype=torch.int32, device=h.device)
        _lib.call("molclr_segment_max_fwd", h.data_ptr(), graph.graph_ptr.data_ptr(), out.data_ptr(),
                  arg.data_ptr(), G, D, dt, _stream(h))
        ctx.save_for_backward(arg)
        ctx.N, ctx.dtype, ctx.dt = N, h.dtype, dt
        return out

    @staticmethod
    def backward(ctx, dout):
        (arg,) = ctx.saved_tensors
        dout = _c(dout.to(torch.float32))
        G, D = dout.shape
        dh = torch.empty(ctx.N, D, dtype=ctx.dtype, device=dout.device)
        _lib.call("molclr_segment_max_bwd", dout.data_ptr(), arg.data_ptr(), dh.data_ptr(), ctx.N, G,
                  D, ctx.dt, _stream(dout))
        return dh, None


class _GCNConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, bias, E1, E2, graph: DeviceGraph):
        _check(x, W, bias, E1, E2)
        x = _c(x)
        N, Din = x.shape
        Dout = W.shape[1]
        # xW with W stored [in, out] (gcn_molclr.py:45,76): B K-major, ldb = Dout
        ctx.h3 = Din == Dout and gcn_h3_ok(N, Din)
        if ctx.h3:  # the same product, also folding max |x| (the h3 weight gradient's scale)
            ctx.xmax = torch.zeros(MAX_SLOT, dtype=torch.float32, device=x.device)
            xw = torch.empty(N, Dout, dtype=torch.float32, device=x.device)
            ws_bytes = _wsq("molclr_gemm_f32_workspace_bytes", N, Dout, Din)
            ws = _ws(ws_bytes, x.device) if ws_bytes else None
            _lib.call("molclr_gemm_f32_bplanes_max", x.data_ptr(),
                      weight_planes(W, Dout, Din, Dout, 1).data_ptr(), xw.data_ptr(), N, Dout,
                      Din, x.stride(0), xw.stride(0), EPI_NONE, None, None, 0,
                      ctx.xmax.data_ptr(), None, None, None, _lib.ptr(ws), ws_bytes, _stream(x))
        else:
            xw = gemm_w(x, W, N, Dout, Din, Din, Dout, False, True)
        out = torch.empty(N, Dout, dtype=torch.float32, device=x.device)
        _lib.call("molclr_gcn_aggregate_fwd", xw.data_ptr(), graph.rowptr.data_ptr(),
                  graph.col.data_ptr(), graph.ecode.data_ptr(), graph.nbr.data_ptr(),
                  E1.data_ptr(), E2.data_ptr(),
                  bias.data_ptr(), out.data_ptr(), N, Dout, _stream(x))
        if _TIMER is not None:
            _TIMER.add("gcn_aggregate_fwd", gine_aggregate_bytes(N, Dout, graph.num_edges))
        ctx.save_for_backward(x, W)
        ctx.graph = graph
        ctx.params = (W, bias, E1, E2)
        return out

    @staticmethod
    def backward(ctx, g):
        x, W = ctx.saved_tensors
        g = _c(g)
        N, Din = x.shape
        Dout = W.shape[1]
        need = ctx.needs_input_grad
        pW, pb, pE1, pE2 = ctx.params
        dxw = torch.empty(N, Dout, dtype=torch.float32, device=g.device)
        sinks = {}
        owned = all(getattr(p, "_molclr_fused_grad", False) and p.grad is not None
                    for p, n in ((pb, need[2]), (pE1, need[3]), (pE2, need[4])) if n)
        for key, p, shape, n in (("b", pb, (Dout,), need[2]), ("e1", pE1, (5, 1), need[3]),
                                 ("e2", pE2, (3, 1), need[4])):
            sinks[key] = _grad_sink(p if owned else None, shape, g.device) if n else (None, 0, None)
        acc = 1 if owned and any(need[2:5]) else 0
        ws_bytes = _wsq("molclr_gcn_aggregate_bwd_workspace_bytes", N, Dout)
        ws = _ws(ws_bytes, g.device)
        _lib.call("molclr_gcn_aggregate_bwd", g.data_ptr(), ctx.graph.rowptr_t.data_ptr(),
                  ctx.graph.col_t.data_ptr(), ctx.graph.nbr_t.data_ptr(),
                  ctx.graph.ecount.data_ptr(), dxw.data_ptr(),
                  _lib.ptr(sinks["e1"][0]), _lib.ptr(sinks["e2"][0]), _lib.ptr(sinks["b"][0]),
                  N, Dout, acc, ws.data_ptr(), ws_bytes, _stream(g))
        db, dE1, dE2 = sinks["b"][2], sinks["e1"][2], sinks["e2"][2]
        dx = dW = None
        if ctx.h3:
            # the executor's h3 order: dxw's row maxima / max, dW (per-tensor
            # scales), dx = dxw W^T (row-wise scales)
            rows = torch.empty(N, dtype=torch.float32, device=g.device)
            dmax = torch.empty(MAX_SLOT, dtype=torch.float32, device=g.device)
            _lib.call("molclr_absmax_rows_f32", dxw.data_ptr(), N, Dout, dxw.stride(0),
                      rows.data_ptr(), dmax.data_ptr(), 0, _stream(g))
            if need[1]:
                buf, a, dW = _grad_sink(pW, (Din, Dout), g.device)
                wsb = _wsq("molclr_linear_wgrad_workspace_bytes", N, Din, Dout)
                wsw = _ws(wsb, g.device)
                _lib.call("molclr_linear_wgrad_h3", x.data_ptr(), ctx.xmax.data_ptr(),
                          dxw.data_ptr(), dmax.data_ptr(), buf.data_ptr(), None, N, Din, Dout,
                          x.stride(0), dxw.stride(0), a, wsw.data_ptr(), wsb, _stream(g))
            if need[0]:
                dx = gemm_h3(dxw, rows, W, Din, Dout, Dout, 0, rowwise=1)
            return dx, dW, db, dE1, dE2, None
        if need[1]:
            # dW[Din,Dout] = x^T dxw
            buf, a, dW = _grad_sink(pW, (Din, Dout), g.device)
            gemm(x, dxw, Din, Dout, N, Din, Dout, True, True, out=buf, accumulate=a)
        if need[0]:
            # dx[N,Din] = dxw W^T : B(k=o, n=i) = W[i, o] (not K-major, ldb = Dout)
            dx = gemm_w(dxw, W, N, Din, Dout, Dout, Dout, False, False)
        return dx, dW, db, dE1, dE2, None


class _L2Normalize(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, eps):
        _check(z)
        z = _c(z)
        rows, D = z.shape
        y = torch.empty_like(z)
        norm = torch.empty(rows, dtype=torch.float32, device=z.device)
        _lib.call("molclr_l2norm_fwd", z.data_ptr(), y.data_ptr(), norm.data_ptr(), rows, D,
                  float(eps), _stream(z))
        ctx.save_for_backward(y, norm)
        ctx.eps = eps
        return y

    @staticmethod
    def backward(ctx, dy):
        y, norm = ctx.saved_tensors
        dy = _c(dy)
        rows, D = y.shape
        dz = torch.empty_like(y)
        _lib.call("molclr_l2norm_bwd", dy.data_ptr(), y.data_ptr(), norm.data_ptr(), dz.data_ptr(),
                  rows, D, float(ctx.eps), _stream(dy))
        return dz, None


# gidx (each local row's global R row) per (n, rank, world, device): built once
# outside any capture (CapturedTrainStep's dry run populates it first)
_GIDX: dict = {}


def _row_index(n, dev, group):
    if group is None:
        key, rank, world = (n, dev.index, 0, 1), 0, 1
    else:
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        key = (n, dev.index, rank, world)
    g = _GIDX.get(key)
    if g is not None:
        return g
    if group is None:
        g = torch.arange(n, dtype=torch.int32, device=dev)
    else:
        from . import distributed as mdist
        g = mdist.global_row_index(n // 2, rank, world, dev)
    if not torch.cuda.is_current_stream_capturing():
        _GIDX[key] = g
    return g


def _ntxent_rows_forward(ctx, rhat, batch_size, temperature, group):
    """NT-Xent over this process's prepared rows rhat (utils/nt_xent.py:47-65
    after the row scaling): the columns (gathered with a group), the row
    logsumexp, the loss; saves what _ntxent_rows_backward needs."""
    dev = rhat.device
    n, C = rhat.shape
    Bl = n // 2
    st = _lib.stream_of(dev)
    if group is None:
        B = Bl
        if batch_size != B:
            raise ValueError(f"NTXentLoss built for batch_size={batch_size} got {B} rows "
                             "(the reference requires full batches, dataset.py:179)")
        cols = rhat
    else:
        import torch.distributed as dist

        from . import distributed as mdist
        B = Bl * dist.get_world_size(group)
        if batch_size != B:
            raise ValueError(f"global batch {B} != NTXentLoss batch_size {batch_size}")
        cols = mdist.gather_rows(rhat, group)
    gidx = _row_index(n, dev, group)
    lse = torch.empty(n, dtype=torch.float32, device=dev)
    loss_rows = torch.empty(n, dtype=torch.float32, device=dev)
    ws_bytes = _wsq("molclr_ntxent_workspace_bytes", n, 2 * B, C)
    ws = _ws(ws_bytes, dev)
    # the GEMM formulations keep S for the backward
    sim_bytes = _wsq("molclr_ntxent_sim_bytes", n, 2 * B, C, -1)
    sim = (torch.empty(sim_bytes // 4, dtype=torch.float32, device=dev) if sim_bytes
           else torch.empty(0, dtype=torch.float32, device=dev))
    _lib.call("molclr_ntxent_fwd_impl", rhat.data_ptr(), gidx.data_ptr(), cols.data_ptr(), n,
              2 * B, C, B, float(temperature), lse.data_ptr(), loss_rows.data_ptr(),
              sim.data_ptr() if sim_bytes else None, ws.data_ptr(), ws_bytes, st, -1)
    if _TIMER is not None:
        _TIMER.add("ntxent", 2.0 * n * 2 * B * C)
    loss = torch.empty((), dtype=torch.float32, device=dev)
    _lib.call("molclr_sum_f32", loss_rows.data_ptr(), loss.data_ptr(), n, st)
    if group is None:
        lse_cols = lse
    else:  # one all-gather carries the row lse and the rank's loss share
        from . import distributed as mdist
        lse_cols, loss = mdist.gather_lse_and_sum(lse, loss, group)
    # tensors through save_for_backward by the caller (autograd's version
    # checks; a retained graph can run backward twice), scalars on ctx
    ctx.ntx = (B, C, float(temperature))
    return loss, (cols, gidx, lse_cols, sim)


def _ntxent_rows_backward(ctx, rhat, gloss, cols, gidx, lse_cols, sim):
    """drhat (this process's rows) from the upstream scalar gradient."""
    B, C, T = ctx.ntx
    dev = rhat.device
    n = rhat.shape[0]
    gloss = gloss.to(torch.float32).contiguous()
    drhat = torch.empty_like(rhat)
    ws_bytes = _wsq("molclr_ntxent_workspace_bytes", n, 2 * B, C)
    ws = _ws(ws_bytes, dev)
    _lib.call("molclr_ntxent_bwd_impl", rhat.data_ptr(), gidx.data_ptr(), cols.data_ptr(),
              lse_cols.data_ptr(), gloss.data_ptr(), n, 2 * B, C, B, T,
              sim.data_ptr() if sim.numel() else None, drhat.data_ptr(), ws.data_ptr(),
              ws_bytes, _lib.stream_of(dev), -1)
    if _TIMER is not None:  # dR = W R (and S again when the forward kept none)
        _TIMER.add("ntxent", (2.0 if sim.numel() else 4.0) * n * 2 * B * C)
    return drhat


class _NTXent(torch.autograd.Function):
    """NT-Xent over this process's rows R = [zj; zi] (utils/nt_xent.py:48).
    With a ``group`` (torch.distributed) the batch is the global one: rows
    are this rank's, columns are gathered (molclr_amd.distributed)."""

    @staticmethod
    def forward(ctx, R, batch_size, temperature, cosine, group):
        _check(R)
        R = _c(R)
        n, C = R.shape
        rhat = torch.empty_like(R)
        norm = torch.empty(n, dtype=torch.float32, device=R.device)
        _lib.call("molclr_ntxent_prep", R.data_ptr(), rhat.data_ptr(), norm.data_ptr(), n, C,
                  int(cosine), _lib.stream_of(R.device))
        loss, kept = _ntxent_rows_forward(ctx, rhat, batch_size, temperature, group)
        ctx.save_for_backward(rhat, norm, *kept)
        ctx.cosine = int(cosine)
        return loss

    @staticmethod
    def backward(ctx, gloss):
        rhat, norm, *kept = ctx.saved_tensors
        n, C = rhat.shape
        drhat = _ntxent_rows_backward(ctx, rhat, gloss, *kept)
        dR = torch.empty_like(rhat)
        _lib.call("molclr_ntxent_prep_bwd", drhat.data_ptr(), rhat.data_ptr(), norm.data_ptr(),
                  dR.data_ptr(), n, C, ctx.cosine, _lib.stream_of(rhat.device))
        return dR, None, None, None, None


class _NTXentPairNormalized(torch.autograd.Function):
    """F.normalize (molclr.py:63-64) and NT-Xent (utils/nt_xent.py:47-65) of a
    paired forward's projections z = [zis; zjs] as one node:
    molclr_ntxent_prep_pair does the row swap to R = [zjs; zis], F.normalize
    and the cosine scaling in one launch (bit-identical to l2_normalize +
    torch.cat + _NTXent's prep), and its backward puts dz straight into z's
    row order."""

    @staticmethod
    def forward(ctx, z, batch_size, temperature, cosine, group, eps):
        _check(z)
        z = _c(z)
        n, C = z.shape
        dev = z.device
        y = torch.empty_like(z)
        rhat = torch.empty_like(z)
        n1 = torch.empty(n, dtype=torch.float32, device=dev)
        n2 = torch.empty(n, dtype=torch.float32, device=dev)
        _lib.call("molclr_ntxent_prep_pair", z.data_ptr(), y.data_ptr(), rhat.data_ptr(),
                  n1.data_ptr(), n2.data_ptr(), n // 2, C, float(eps), int(cosine),
                  _lib.stream_of(dev))
        loss, kept = _ntxent_rows_forward(ctx, rhat, batch_size, temperature, group)
        ctx.save_for_backward(y, rhat, n1, n2, *kept)
        ctx.cosine, ctx.eps = int(cosine), float(eps)
        return loss

    @staticmethod
    def backward(ctx, gloss):
        y, rhat, n1, n2, *kept = ctx.saved_tensors
        n, C = rhat.shape
        drhat = _ntxent_rows_backward(ctx, rhat, gloss, *kept)
        dz = torch.empty_like(rhat)
        _lib.call("molclr_ntxent_prep_pair_bwd", drhat.data_ptr(), rhat.data_ptr(), n2.data_ptr(),
                  y.data_ptr(), n1.data_ptr(), dz.data_ptr(), n // 2, C, ctx.eps, ctx.cosine,
                  _lib.stream_of(rhat.device))
        return dz, None, None, None, None, None


GIN_PARAMS_PER_LAYER = 8  # mlp0.W, mlp0.b, mlp2.W, mlp2.b, edge_emb1, edge_emb2, bn.W, bn.b


class _GINEncoder(torch.autograd.Function):
    """The whole GINet node-embedding stack (ginet_molclr.py:98-111) through
    molclr_gin_encoder_fwd / _bwd (encoder.hip): the same kernels as the
    per-op path in the same order, one host call each way.
    params: x_embedding1, x_embedding2, then per layer GIN_PARAMS_PER_LAYER."""

    @staticmethod
    def forward(ctx, x_idx, graph: DeviceGraph, bns, dtype, *params):
        _check(x_idx, *params)
        L = len(bns)
        D = params[0].shape[1]
        x_idx = _c(x_idx.to(torch.long))
        N = graph.num_nodes
        training = bool(bns[0].training)
        enc = _lib.GinEncoder()
        enc.num_layer, enc.training, enc.dim = L, int(training), D
        enc.dtype = dtype
        # fp32: the GEMM form ops._MLP would use on these shapes (identical kernels)
        h3 = dtype == _lib.DTYPE_F32 and h3_ok(N, D)
        kind = "h3" if h3 and H3_FORWARD else "x6"
        kind_t = "h3" if h3 else "x6"
        enc.fp32_gemm = (1 | (2 if H3_FORWARD else 0)) if h3 else 0
        enc.status = graph.status.data_ptr()  # out-of-vocabulary atoms: MOLCLR_STATUS_ATOM_RANGE
        enc.n_atom, enc.n_chiral = params[0].shape[0], params[1].shape[0]
        enc.momentum, enc.eps = float(bns[0].momentum), float(bns[0].eps)
        enc.x_embedding1, enc.x_embedding2 = params[0].data_ptr(), params[1].data_ptr()
        for l in range(L):
            W0, b0, W2, b2, E1, E2, g, b = params[2 + GIN_PARAMS_PER_LAYER * l:
                                                  2 + GIN_PARAMS_PER_LAYER * (l + 1)]
            bn = bns[l]
            enc.mlp0_weight[l], enc.mlp0_bias[l] = W0.data_ptr(), b0.data_ptr()
            enc.mlp2_weight[l], enc.mlp2_bias[l] = W2.data_ptr(), b2.data_ptr()
            enc.edge_embedding1[l], enc.edge_embedding2[l] = E1.data_ptr(), E2.data_ptr()
            enc.bn_weight[l], enc.bn_bias[l] = g.data_ptr(), b.data_ptr()
            enc.bn_running_mean[l] = bn.running_mean.data_ptr()
            enc.bn_running_var[l] = bn.running_var.data_ptr()
            nbt = bn.num_batches_tracked
            enc.bn_num_batches_tracked[l] = nbt.data_ptr() if training and nbt is not None else None
            twoD = W0.shape[0]
            # the same planes (and cache entries) ops.linear_fwd / linear_bwd use
            enc.mlp0_planes[l] = weight_planes(W0, twoD, D, D, 0, kind).data_ptr()
            enc.mlp0_planes_t[l] = weight_planes(W0, D, twoD, D, 1, kind_t).data_ptr()
            enc.mlp2_planes[l] = weight_planes(W2, D, twoD, twoD, 0, kind).data_ptr()
            enc.mlp2_planes_t[l] = weight_planes(W2, twoD, D, twoD, 1, kind_t).data_ptr()
        dev = x_idx.device
        arena_bytes = _wsq("molclr_gin_encoder_arena_bytes", L, N, D, dtype)
        arena = torch.empty(max(arena_bytes // 4, 1), dtype=torch.float32, device=dev)
        ws_bytes = _wsq("molclr_gin_encoder_workspace_bytes", L, N, D, dtype)
        ws = _ws(ws_bytes, dev)
        h = torch.empty(N, D, dtype=TORCH_DTYPE[dtype], device=dev)
        gc = graph.cstruct()
        _lib.call("molclr_gin_encoder_fwd", ctypes.addressof(enc), x_idx.data_ptr(),
                  ctypes.addressof(gc), h.data_ptr(), arena.data_ptr(), arena_bytes,
                  ws.data_ptr(), ws_bytes, _stream(x_idx))
        if _TIMER is not None:
            es = 2 if dtype == _lib.DTYPE_BF16 else 4
            # the h3 forward's aggregation also stores its row maxima
            rmb = _wsq("molclr_rowmax_bytes", N, D) if (enc.fp32_gemm & 2) else 0
            for _ in range(L):
                _TIMER.add("gine_aggregate_fwd",
                           gine_aggregate_bytes(N, D, graph.num_edges, es) + rmb)
                _TIMER.add("gemm_f32", 2 * 2.0 * N * D * (2 * D))
        ctx.enc, ctx.graph, ctx.arena, ctx.arena_bytes = enc, graph, arena, arena_bytes
        ctx.x_idx, ctx.params, ctx.training = x_idx, params, training
        return h

    @staticmethod
    def backward(ctx, dh):
        if not ctx.training:
            raise NotImplementedError("molclr_amd: backward through eval-mode BatchNorm")
        dtype = int(ctx.enc.dtype)
        dh = _c(dh.to(TORCH_DTYPE[dtype]))
        params = ctx.params
        L = ctx.enc.num_layer
        N, D = dh.shape
        owned = all(getattr(p, "_molclr_fused_grad", False) and p.grad is not None
                    for p in params)
        if owned:  # FusedAdam: add straight into the flat gradient buffer
            bufs = [p.grad for p in params]
            ret = [None] * len(params)
        else:
            bufs = [torch.zeros_like(p) for p in params]
            ret = bufs
        gr = _lib.GinEncoderGrads()
        gr.x_embedding1, gr.x_embedding2 = bufs[0].data_ptr(), bufs[1].data_ptr()
        names = ("mlp0_weight", "mlp0_bias", "mlp2_weight", "mlp2_bias", "edge_embedding1",
                 "edge_embedding2", "bn_weight", "bn_bias")
        for l in range(L):
            for j, nm in enumerate(names):
                getattr(gr, nm)[l] = bufs[2 + GIN_PARAMS_PER_LAYER * l + j].data_ptr()
        ws_bytes = _wsq("molclr_gin_encoder_workspace_bytes", L, N, D, dtype)
        ws = _ws(ws_bytes, dh.device)
        gc = ctx.graph.cstruct()
        hook = _grad_events(gr, L, owned)
        _lib.call("molclr_gin_encoder_bwd", ctypes.addressof(ctx.enc), ctypes.addressof(gr),
                  ctx.x_idx.data_ptr(), ctypes.addressof(gc), dh.data_ptr(), ctx.arena.data_ptr(),
                  ctx.arena_bytes, ws.data_ptr(), ws_bytes, _stream(dh))
        if hook is not None:
            hook.encoder_backward_enqueued()
        if _TIMER is not None:
            for _ in range(L):
                _TIMER.add("gemm_f32", 4 * 2.0 * N * D * (2 * D))
        ctx.arena = None
        return (None, None, None, None, *ret)


GCN_PARAMS_PER_LAYER = 6  # weight, bias, edge_emb1, edge_emb2, bn.W, bn.b


class _GCNEncoder(torch.autograd.Function):
    """GCN's node-embedding stack (gcn_molclr.py:140-151) through
    molclr_gcn_encoder_fwd / _bwd (encoder.hip): the per-op path's kernels in
    its order, one host call each way.
    params: x_embedding1, x_embedding2, then per layer GCN_PARAMS_PER_LAYER."""

    @staticmethod
    def forward(ctx, x_idx, graph: DeviceGraph, bns, *params):
        _check(x_idx, *params)
        L = len(bns)
        D = params[0].shape[1]
        x_idx = _c(x_idx.to(torch.long))
        N = graph.num_nodes
        training = bool(bns[0].training)
        enc = _lib.GcnEncoder()
        enc.num_layer, enc.training, enc.dim = L, int(training), D
        enc.n_atom, enc.n_chiral = params[0].shape[0], params[1].shape[0]
        enc.momentum, enc.eps = float(bns[0].momentum), float(bns[0].eps)
        enc.x_embedding1, enc.x_embedding2 = params[0].data_ptr(), params[1].data_ptr()
        h3 = gcn_h3_ok(N, D)  # the form _GCNConv uses on these shapes
        enc.fp32_gemm = int(h3)
        enc.status = graph.status.data_ptr()
        for l in range(L):
            W, b, E1, E2, g, bb = params[2 + GCN_PARAMS_PER_LAYER * l:
                                         2 + GCN_PARAMS_PER_LAYER * (l + 1)]
            bn = bns[l]
            enc.weight[l], enc.bias[l] = W.data_ptr(), b.data_ptr()
            enc.edge_embedding1[l], enc.edge_embedding2[l] = E1.data_ptr(), E2.data_ptr()
            enc.bn_weight[l], enc.bn_bias[l] = g.data_ptr(), bb.data_ptr()
            enc.bn_running_mean[l] = bn.running_mean.data_ptr()
            enc.bn_running_var[l] = bn.running_var.data_ptr()
            nbt = bn.num_batches_tracked
            enc.bn_num_batches_tracked[l] = nbt.data_ptr() if training and nbt is not None else None
            # the planes (and cache entries) _GCNConv's gemm_w calls use
            enc.weight_planes[l] = weight_planes(W, D, D, D, 1).data_ptr()
            enc.weight_planes_t[l] = weight_planes(W, D, D, D, 0, "h3" if h3 else "x6").data_ptr()
        dev = x_idx.device
        arena_bytes = _wsq("molclr_gcn_encoder_arena_bytes", L, N, D)
        arena = torch.empty(max(arena_bytes // 4, 1), dtype=torch.float32, device=dev)
        ws_bytes = _wsq("molclr_gcn_encoder_workspace_bytes", L, N, D)
        ws = _ws(ws_bytes, dev)
        h = torch.empty(N, D, dtype=torch.float32, device=dev)
        gc = graph.cstruct()
        _lib.call("molclr_gcn_encoder_fwd", ctypes.addressof(enc), x_idx.data_ptr(),
                  ctypes.addressof(gc), h.data_ptr(), arena.data_ptr(), arena_bytes,
                  ws.data_ptr(), ws_bytes, _stream(x_idx))
        if _TIMER is not None:
            for _ in range(L):
                _TIMER.add("gemm_f32", 2.0 * N * D * D)
                # the GCN scatter-add moves the same compulsory bytes as GINE's
                _TIMER.add("gcn_aggregate_fwd", gine_aggregate_bytes(N, D, graph.num_edges))
        ctx.enc, ctx.graph, ctx.arena, ctx.arena_bytes = enc, graph, arena, arena_bytes
        ctx.x_idx, ctx.params, ctx.training = x_idx, params, training
        return h

    @staticmethod
    def backward(ctx, dh):
        if not ctx.training:
            raise NotImplementedError("molclr_amd: backward through eval-mode BatchNorm")
        dh = _c(dh)
        params = ctx.params
        L = ctx.enc.num_layer
        N, D = dh.shape
        owned = all(getattr(p, "_molclr_fused_grad", False) and p.grad is not None
                    for p in params)
        if owned:  # FusedAdam: add straight into the flat gradient buffer
            bufs = [p.grad for p in params]
            ret = [None] * len(params)
        else:
            bufs = [torch.zeros_like(p) for p in params]
            ret = bufs
        gr = _lib.GcnEncoderGrads()
        gr.x_embedding1, gr.x_embedding2 = bufs[0].data_ptr(), bufs[1].data_ptr()
        names = ("weight", "bias", "edge_embedding1", "edge_embedding2", "bn_weight", "bn_bias")
        for l in range(L):
            for j, nm in enumerate(names):
                getattr(gr, nm)[l] = bufs[2 + GCN_PARAMS_PER_LAYER * l + j].data_ptr()
        ws_bytes = _wsq("molclr_gcn_encoder_workspace_bytes", L, N, D)
        ws = _ws(ws_bytes, dh.device)
        gc = ctx.graph.cstruct()
        hook = _grad_events(gr, L, owned)
        _lib.call("molclr_gcn_encoder_bwd", ctypes.addressof(ctx.enc), ctypes.addressof(gr),
                  ctx.x_idx.data_ptr(), ctypes.addressof(gc), dh.data_ptr(), ctx.arena.data_ptr(),
                  ctx.arena_bytes, ws.data_ptr(), ws_bytes, _stream(dh))
        if hook is not None:
            hook.encoder_backward_enqueued()
        if _TIMER is not None:
            for _ in range(L):
                _TIMER.add("gemm_f32", 2 * 2.0 * N * D * D)
        ctx.arena = None
        return (None, None, None, *ret)


def gcn_encoder(x_idx, graph, bns, params):
    """GCN.encode through the encoder executor (see _GCNEncoder)."""
    return _GCNEncoder.apply(x_idx, graph, bns, *params)


DTYPES = {"fp32": _lib.DTYPE_F32, "bf16": _lib.DTYPE_BF16}
TORCH_DTYPE = {_lib.DTYPE_F32: torch.float32, _lib.DTYPE_BF16: torch.bfloat16}


def gin_encoder(x_idx, graph, bns, params, precision: str = "fp32"):
    """GINet.encode through the encoder executor (see _GINEncoder); precision
    "bf16" runs the c5 configuration's bf16 storage / bf16 MFMA path and
    returns bf16 node embeddings."""
    return _GINEncoder.apply(x_idx, graph, bns, DTYPES[precision], *params)


# public functional API -------------------------------------------------------
def atom_embed(x_idx, X1, X2, status=None):
    """ginet_molclr.py:103.  An out-of-vocabulary atom gives a NaN row and
    sets MOLCLR_STATUS_ATOM_RANGE in ``status`` (e.g. the graph's word)."""
    return _AtomEmbed.apply(x_idx, X1, X2, status)


def gine_aggregate(h, E1, E2, graph, Ec=None):
    """Ec: this layer's [15, D] slice of edge_tables_combine (computed here if None)."""
    return _GINEAggregate.apply(h, E1, E2, graph, Ec)


def gin_mlp(x, W1, b1, W2, b2, side=False):
    return _MLP.apply(x, W1, b1, W2, b2, side)


def projection_head(x, W1, b1, W2, b2, side=False):
    """out_lin; ``side``: weight gradients on the side stream (join_side)."""
    return _MLP.apply(x, W1, b1, W2, b2, side)


def linear(x, W, b, side=False):
    return _Linear.apply(x, W, b, side)


def batch_norm(z, bn: torch.nn.BatchNorm1d, relu: bool):
    training = bn.training or not bn.track_running_stats
    update = bn.training and bn.track_running_stats
    nbt = bn.num_batches_tracked if update and bn.num_batches_tracked is not None else None
    if bn.momentum is None:
        if nbt is not None:
            nbt.add_(1)  # cumulative average needs the count now (torch semantics)
            momentum = 1.0 / float(nbt.item())
            nbt = None
        else:
            momentum = 0.0
    else:
        momentum = bn.momentum  # num_batches_tracked += 1 happens in the stats kernel
    return _BatchNorm.apply(z, bn.weight, bn.bias,
                            bn.running_mean if bn.track_running_stats else None,
                            bn.running_var if bn.track_running_stats else None,
                            training, momentum, bn.eps, relu, nbt)


def segment_pool(h, graph, mode: str):
    """global_mean_pool / global_add_pool / global_max_pool over graph_ptr."""
    if mode == "max":
        return _SegmentMax.apply(h, graph)
    if mode not in POOL_MODES:
        raise ValueError(f"pool '{mode}' is not supported by molclr_amd (mean, add, max)")
    return _SegmentPool.apply(h, graph, POOL_MODES[mode])


def gcn_conv(x, W, bias, E1, E2, graph):
    return _GCNConv.apply(x, W, bias, E1, E2, graph)


def l2_normalize(z, eps: float = 1e-12):
    return _L2Normalize.apply(z, eps)


def nt_xent(zis, zjs, batch_size, temperature, use_cosine_similarity=True, group=None):
    """NTXentLoss.forward(zis, zjs): R = [zjs; zis] (utils/nt_xent.py:48)."""
    _check(zis, zjs)
    return _NTXent.apply(torch.cat([zjs, zis], 0), batch_size, temperature,
                         bool(use_cosine_similarity), group)


def nt_xent_pair(z, batch_size, temperature, use_cosine_similarity=True, group=None):
    """NT-Xent of a paired forward's projections z = [zis; zjs] (one tensor)."""
    _check(z)
    B = z.shape[0] // 2
    return _NTXent.apply(torch.cat([z[B:], z[:B]], 0), batch_size, temperature,
                         bool(use_cosine_similarity), group)


def nt_xent_pair_normalized(z, batch_size, temperature, use_cosine_similarity=True, group=None,
                            eps: float = 1e-12):
    """nt_xent_pair(l2_normalize(z)) as one autograd node (one prep launch
    each way instead of l2norm + cat + prep and their backwards; the same
    values bit for bit)."""
    _check(z)
    return _NTXentPairNormalized.apply(z, batch_size, temperature, bool(use_cosine_similarity),
                                       group, eps)
