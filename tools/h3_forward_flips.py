"""Elementwise accuracy of the forward product z1 = agg W0^T + b (GIN MLP lin1,
models/ginet_molclr.py:19-23 at c2: 30,556 x 300 -> 600) under each fp32 GEMM
form, against fp64:

- ``fp32 cpu``: torch's CPU sgemm -- the reference's own fp32 path;
- ``x6``: six split-bf16 MFMAs (the product forward);
- ``h3 rows``: three fp16 MFMAs, A scaled per row (MOLCLR_H3_FORWARD=1);
- ``h3 tensor``: three fp16 MFMAs, A scaled by its tensor max.

For each: the error relative to the dot product's magnitude sum
(|agg| |W0|^T + |b|), and the ReLU decisions (z > 0) that differ from fp64's.
Inputs: rows of N(0, 1) with a log-normal row scale (sigma 1, so row maxima
span ~5 orders), W0 / b as nn.Linear initialises them.

    python tools/h3_forward_flips.py [rows]
"""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from molclr_amd import _lib, ops  # noqa: E402
from molclr_amd._lib import EPI_BIAS  # noqa: E402


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 30556
    K, N = 300, 600
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    agg = torch.randn(M, K, generator=g) * torch.exp(torch.randn(M, 1, generator=g))
    bound = 1.0 / K ** 0.5
    W = (torch.rand(N, K, generator=g) * 2 - 1) * bound
    b = (torch.rand(N, generator=g) * 2 - 1) * bound
    z64 = agg.double() @ W.double().T + b.double()
    mag = agg.double().abs() @ W.double().abs().T + b.double().abs()
    out = {"fp32 cpu": (agg @ W.T + b).double()}

    A, Wd, bd = agg.to(dev), W.to(dev), b.to(dev)
    st = _lib.stream_of(dev)
    lib = _lib.load()
    out["x6"] = ops.gemm_w(A, Wd, M, N, K, K, K, False, False, EPI_BIAS, bias=bd).double().cpu()
    rmax = torch.empty(M, device=dev)
    slot = torch.zeros(ops.MAX_SLOT, device=dev)
    lib.molclr_absmax_rows_f32(A.data_ptr(), M, K, K, rmax.data_ptr(), slot.data_ptr(), 1, st)
    out["h3 rows"] = ops.gemm_h3(A, rmax, Wd, N, K, K, 0, EPI_BIAS, bias=bd,
                                 rowwise=1).double().cpu()
    out["h3 tensor"] = ops.gemm_h3(A, ops.absmax(A), Wd, N, K, K, 0, EPI_BIAS,
                                   bias=bd).double().cpu()
    torch.cuda.synchronize()

    pos64 = z64 > 0
    near = (z64.abs() < 1e-4 * mag)  # decisions within 1e-4 of the magnitude sum
    for name, z in out.items():
        e = (z - z64).abs() / mag
        flips = int(((z > 0) != pos64).sum())
        print(json.dumps({
            "form": name, "rows": M,
            "err_rel_max": float(e.max()), "err_rel_mean": float(e.mean()),
            "err_rel_p999": float(torch.quantile(e.flatten()[::7].float(), 0.999)),
            "relu_flips_vs_fp64": flips,
            "near_zero_elems": int(near.sum()),
            "err_rel_max_near_zero": float(e[near].max()) if near.any() else 0.0,
        }), flush=True)


if __name__ == "__main__":
    main()
