"""Diagnostic (GPU box): per-stage gradient comparison of the HIP GINet/GCN
against the oracle in fp32 and fp64.  Prints, for every layer, the relative
error of d(layer input), d(conv output), d(BN output), and every parameter
gradient, for mine-vs-fp64 and oracle32-vs-fp64."""
import copy
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from molclr_amd import ops  # noqa: E402
from molclr_amd.dataset import SyntheticPairBatches  # noqa: E402
from molclr_amd.gcn_molclr import GCN  # noqa: E402
from molclr_amd.ginet_molclr import GINet  # noqa: E402
from oracle.reference_cpu import RefGCN, RefGINet  # noqa: E402


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return (a - b).norm().item() / max(b.norm().item(), 1e-30)


def capture_ref(model, store):
    for l, conv in enumerate(model.gnns):
        def pre(mod, args, l=l):
            args[0].retain_grad()
            store[f"in{l}"] = args[0]

        def post(mod, args, out, l=l):
            out.retain_grad()
            store[f"conv{l}"] = out
        conv.register_forward_pre_hook(pre)
        conv.register_forward_hook(post)
    for l, bn in enumerate(model.batch_norms):
        def post(mod, args, out, l=l):
            out.retain_grad()
            store[f"bn{l}"] = out
        bn.register_forward_hook(post)


def run(kind, L, D, B):
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    R = RefGINet if kind == "gin" else RefGCN
    P = GINet if kind == "gin" else GCN
    ref = R(L, D, 512)
    ref64 = copy.deepcopy(ref).double()
    mine = P(L, D, 512)
    mine.load_state_dict(ref.state_dict())
    mine = mine.to(dev)
    bi, _ = SyntheticPairBatches(B, seed=11).next()

    s32, s64, sm = {}, {}, {}
    capture_ref(ref, s32)
    capture_ref(ref64, s64)
    # product: wrap the op entry points to retain intermediate grads
    orig = {}
    counters = {"in": 0, "conv": 0, "bn": 0}

    def wrap(name, key, fn, arg_index=None):
        def f(*a, **k):
            if arg_index is not None:
                x = a[arg_index]
                if x.requires_grad:
                    x.retain_grad()
                sm[f"in{counters['in']}"] = x
                counters["in"] += 1
            out = fn(*a, **k)
            if key:
                out.retain_grad()
                sm[f"{key}{counters[key]}"] = out
                counters[key] += 1
            return out
        return f
    if kind == "gin":
        orig["gine_aggregate"] = ops.gine_aggregate
        ops.gine_aggregate = wrap("gine_aggregate", None, ops.gine_aggregate, arg_index=0)
        orig["gin_mlp"] = ops.gin_mlp
        ops.gin_mlp = wrap("gin_mlp", "conv", ops.gin_mlp)
    else:
        orig["gcn_conv"] = ops.gcn_conv
        ops.gcn_conv = wrap("gcn_conv", "conv", ops.gcn_conv, arg_index=0)
    orig["batch_norm"] = ops.batch_norm
    ops.batch_norm = wrap("batch_norm", "bn", ops.batch_norm)

    h_r, o_r = ref(bi)
    h_6, o_6 = ref64(bi)
    h_m, o_m = mine(bi.to(dev))
    for k, v in orig.items():
        setattr(ops, k, v)
    torch.manual_seed(3)
    w1, w2 = torch.randn_like(h_r), torch.randn_like(o_r)
    ((h_r * w1).sum() + (o_r * w2).sum()).backward()
    ((h_6 * w1.double()).sum() + (o_6 * w2.double()).sum()).backward()
    ((h_m * w1.to(dev)).sum() + (o_m * w2.to(dev)).sum()).backward()
    print(f"== {kind} L={L} D={D} B={B}  fwd h: mine {rel(h_m, h_6):.2e} ref32 {rel(h_r, h_6):.2e}")
    for l in range(L):
        for key in (f"bn{l}", f"conv{l}", f"in{l}"):
            a, b, c = sm.get(key), s32.get(key), s64.get(key)
            if a is None or a.grad is None or c is None or c.grad is None:
                print(f"   {key}: missing")
                continue
            print(f"   d{key:6s} mine {rel(a.grad, c.grad):.2e}  ref32 {rel(b.grad, c.grad):.2e}"
                  f"   fwd mine {rel(a, c):.2e}")
    g6 = dict(ref64.named_parameters())
    g3 = dict(ref.named_parameters())
    for n, p in mine.named_parameters():
        print(f"   {n:36s} mine {rel(p.grad, g6[n].grad):.2e}  ref32 {rel(g3[n].grad, g6[n].grad):.2e}"
              f"  mine-vs-ref32 {rel(p.grad, g3[n].grad):.2e}")


if __name__ == "__main__":
    run("gin", 3, 128, 64)
    run("gcn", 3, 128, 64)
    run("gin", 2, 16, 4)
