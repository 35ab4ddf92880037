"""Check every molclr_gemm_f32 call of one training step against float64.

Runs step 0 of the 3-step training test (GIN 3x128, B=64) with each GEMM
implementation, recording each call's operands; reports per call the norm-wise
and max elementwise error against a float64 product of the same fp32 operands.

    python tools/debug_gemm_calls.py
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from molclr_amd import _lib, ops  # noqa: E402
from molclr_amd.dataset import SyntheticPairBatches  # noqa: E402
from molclr_amd.nt_xent import NTXentLoss  # noqa: E402
from molclr_amd.optim import FusedAdam  # noqa: E402
from oracle.reference_cpu import RefGINet  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    from molclr_amd.ginet_molclr import GINet
    lib = _lib.load()
    torch.manual_seed(1)
    state = RefGINet(3, 128, 512).state_dict()
    xi, xj = SyntheticPairBatches(64, seed=21).next()
    orig = ops.gemm
    grads = {}
    for impl in (0, 1, 4):
        lib.molclr_gemm_set_impl(impl)
        calls = []

        def rec(A, B, M, N, K, lda, ldb, ak, bk, epi=0, bias=None, aux=None, out=None,
                accumulate=0):
            prev = out.clone() if (out is not None and accumulate) else None
            res = orig(A, B, M, N, K, lda, ldb, ak, bk, epi, bias, aux, out, accumulate)
            calls.append((A.clone(), B.clone(), M, N, K, lda, ldb, ak, bk, epi, bias, aux,
                          prev, res.clone()))
            return res

        ops.gemm = rec
        mine = GINet(3, 128, 512)
        mine.load_state_dict(state)
        mine = mine.to(dev)
        opt = FusedAdam(mine.parameters(), 5e-4, weight_decay=1e-5)
        crit = NTXentLoss(dev, 64, 0.1, True)
        opt.zero_grad()
        _, zi = mine(xi.to(dev))
        _, zj = mine(xj.to(dev))
        loss = crit(ops.l2_normalize(zi), ops.l2_normalize(zj))
        loss.backward()
        torch.cuda.synchronize()
        ops.gemm = orig
        print(f"impl{impl}: {len(calls)} gemm calls, loss {loss.item():.7f}")
        grads[impl] = {n: p.grad.detach().double().cpu() for n, p in mine.named_parameters()}
        # guard bands: rerun every call into a buffer with NaN-free sentinels around C
        # and around the split-K workspace
        bad = 0
        for (A, B, M, N, K, lda, ldb, ak, bk, epi, bias, aux, prev, res) in calls:
            G = 4096
            big = torch.full((G + M * N + G,), 12345.0, device=dev)
            outv = big[G:G + M * N].view(M, N)
            if prev is not None:
                outv.copy_(prev)
            wsb = ops._wsq("molclr_gemm_f32_workspace_bytes", M, N, K)
            wsbig = torch.full((G + (wsb + 3) // 4 + G,), 777.0, device=dev)
            e = epi | (16 if prev is not None else 0)
            _lib.call("molclr_gemm_f32", A.data_ptr(), B.data_ptr(), outv.data_ptr(), M, N, K,
                      lda, ldb, N, int(ak), int(bk), e, _lib.ptr(bias), _lib.ptr(aux),
                      aux.stride(0) if aux is not None else 0, wsbig[G:].data_ptr(), wsb,
                      _lib.stream_of(dev))
            torch.cuda.synchronize()
            okc = bool((big[:G] == 12345.0).all() and (big[G + M * N:] == 12345.0).all())
            okw = bool((wsbig[:G] == 777.0).all() and (wsbig[G + (wsb + 3) // 4:] == 777.0).all())
            same = bool(torch.equal(outv, res[:M, :N]))
            if not (okc and okw and same):
                bad += 1
                print(f"  GUARD M{M} N{N} K{K} ak{ak} bk{bk}: C guards {okc} ws guards {okw} "
                      f"rerun identical {same}")
        print(f"  guard check: {bad} bad calls")
        for (A, B, M, N, K, lda, ldb, ak, bk, epi, bias, aux, prev, res) in calls:
            Ad = A.double().cpu().flatten()
            Bd = B.double().cpu().flatten()
            idx_m = torch.arange(M)[:, None]
            idx_k = torch.arange(K)[None, :]
            Am = Ad[(idx_k * lda + idx_m) if ak else (idx_m * lda + idx_k)]
            idx_k2 = torch.arange(K)[:, None]
            idx_n = torch.arange(N)[None, :]
            Bm = Bd[(idx_k2 * ldb + idx_n) if bk else (idx_n * ldb + idx_k2)]
            ref = Am @ Bm
            e = epi & 15
            if e in (1, 2):
                ref = ref + bias.double().cpu()
            if e == 2:
                ref = ref.clamp(min=0)
            if e == 3:
                ref = ref * (aux.double().cpu()[:M, :N] > 0)
            if prev is not None:
                ref = ref + prev.double().cpu()
            out = res.double().cpu()[:M, :N]
            err = (out - ref).norm().item() / max(ref.norm().item(), 1e-30)
            mx = (out - ref).abs().max().item()
            scale = (Am.abs() @ Bm.abs()).max().item()
            flag = " <<<" if err > 1e-5 else ""
            if err > 1e-6:
                print(f"  M{M} N{N} K{K} ak{ak} bk{bk} epi{epi} acc{prev is not None}: rel "
                      f"{err:.2e} max {mx:.2e} (scale {scale:.2e}){flag}")
    for n in grads[0]:
        a, b = grads[0][n], grads[1][n]
        d = ((a - b).norm() / max(b.norm().item(), 1e-30)).item()
        if d > 1e-5:
            print(f"grad {n}: impl0 vs impl1 rel diff {d:.2e}")


if __name__ == "__main__":
    main()
