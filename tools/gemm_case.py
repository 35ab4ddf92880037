"""Run one GEMM shape of the c2 / c5 step repeatedly (for rocprofv3 PMC passes).

    python tools/gemm_case.py CASE [reps] [impl] [--time]

CASE: qb_lin1 qb_lin2 qb_dz1 qb_dagg wb_dW2 wb_dW0 (bf16, c5 shapes, 55k rows)
      q6_lin1 q6_lin2 q6_dz1 q6_dagg w6_dW2 w6_dW1 (fp32 split-bf16, c2, 30.5k rows)
      h3_lin1 h3_dz1 h3_lin2 h3_dagg w6h_dW2 w6h_dW1 (fp32 via three fp16 MFMAs: the c2 step)
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from molclr_amd import _lib, ops  # noqa: E402
from molclr_amd._lib import EPI_BIAS, EPI_BIAS_RELU, EPI_NONE, EPI_RELU_MASK  # noqa: E402


def main():
    case = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    variant = int(sys.argv[3]) if len(sys.argv) > 3 else -1
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    st = _lib.stream_of(dev)
    torch.manual_seed(0)
    bf16 = case[:2] in ("qb", "wb")
    M = 55342 if bf16 else 30556
    D = 512 if bf16 else 300
    H = 2 * D
    dt = torch.bfloat16 if bf16 else torch.float32
    X = {n: torch.randn(M, c, device=dev).to(dt) for n, c in (("agg", D), ("a1", H), ("dz", D),
                                                             ("dz1", H))}
    W0 = torch.randn(H, D, device=dev) * 0.05
    W2 = torch.randn(D, H, device=dev) * 0.05
    b0, b2 = torch.randn(H, device=dev), torch.randn(D, device=dev)
    if bf16:
        p = {"lin1": (ops.weight_planes(W0, H, D, D, 0), "agg", H, D, EPI_BIAS_RELU, b0, None),
             "lin2": (ops.weight_planes(W2, D, H, H, 0), "a1", D, H, EPI_BIAS, b2, None),
             "dz1": (ops.weight_planes(W2, H, D, H, 1), "dz", H, D, EPI_RELU_MASK, None, "a1"),
             "dagg": (ops.weight_planes(W0, D, H, D, 1), "dz1", D, H, EPI_NONE, None, None)}
        if case.startswith("qb"):
            P, a, N, K, epi, bias, aux = p[case[3:]]
            C = torch.empty(M, N, dtype=dt, device=dev)
            auxt = X[aux] if aux else None
            fn = lambda: lib.molclr_gemm_bf16_impl(X[a].data_ptr(), P.data_ptr(), C.data_ptr(), M, N,  # noqa: E731
                                                   K, K, N, epi, _lib.ptr(bias), _lib.ptr(auxt),
                                                   N if aux else 0, st, variant)
        else:
            dy, x, n_out, n_in = (X["dz"], X["a1"], D, H) if case == "wb_dW2" else (X["dz1"], X["agg"], H, D)
            wsb = lib.molclr_linear_wgrad_bf16_workspace_bytes(M, n_out, n_in)
            ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
            dW, db = torch.empty(n_out, n_in, device=dev), torch.empty(n_out, device=dev)
            fn = lambda: lib.molclr_linear_wgrad_bf16_impl(dy.data_ptr(), x.data_ptr(), dW.data_ptr(),  # noqa: E731
                                                           db.data_ptr(), M, n_out, n_in, n_out, n_in,
                                                           0, ws.data_ptr(), wsb, st, variant)
    else:
        t = max(variant, 0)  # molclr_gemm_f32_bplanes_tile: 9 q6, 10 q7, 0 automatic
        # h3 inputs: row maxima (one partial array) and max slots, as the step has them
        rdz = torch.empty(M, device=dev)
        rdz1 = torch.empty(M, device=dev)
        ragg = torch.empty(M, device=dev)
        bits = torch.randint(-2**31, 2**31 - 1, ((H + 31) // 32, M), dtype=torch.int32, device=dev)
        smax = {n: torch.zeros(ops.MAX_SLOT, device=dev) for n in X}
        ra1 = torch.empty(M, device=dev)
        for n, r in (("dz", rdz), ("dz1", rdz1), ("agg", ragg), ("a1", ra1)):
            lib.molclr_absmax_rows_f32(X[n].data_ptr(), M, X[n].shape[1], X[n].shape[1],
                                       r.data_ptr(), smax[n].data_ptr(), 1, st)
        for n in ("agg", "a1"):
            ops.absmax(X[n], out=smax[n])
        Wg0 = torch.nn.Parameter(W0.clone())
        Wg2 = torch.nn.Parameter(W2.clone())
        bg0 = torch.nn.Parameter(b0.clone())
        bg2 = torch.nn.Parameter(b2.clone())
        cases = {"q6_lin1": lambda: ops.gemm_w(X["agg"], W0, M, H, D, D, D, False, False,
                                               EPI_BIAS_RELU, bias=b0, tile=t),
                 "q6_lin2": lambda: ops.gemm_w(X["a1"], W2, M, D, H, H, H, False, False,
                                               EPI_BIAS, bias=b2, tile=t),
                 "q6_dz1": lambda: ops.gemm_w(X["dz"], W2, M, H, D, D, H, False, True,
                                              EPI_RELU_MASK, aux=X["a1"], tile=t),
                 "q6_dagg": lambda: ops.gemm_w(X["dz1"], W0, M, D, H, H, D, False, True, tile=t),
                 # the step's dz1 takes its ReLU mask from lin1's bits (as it does there)
                 "h3_dz1": lambda: ops.gemm_h3(X["dz"], rdz, W2, H, D, H, 1, EPI_RELU_MASK,
                                               rowwise=1, mask_bits=bits),
                 "h3_dz1_aux": lambda: ops.gemm_h3(X["dz"], rdz, W2, H, D, H, 1, EPI_RELU_MASK,
                                                   aux=X["a1"], rowwise=1),
                 "h3_dagg": lambda: ops.gemm_h3(X["dz1"], rdz1, W0, D, H, D, 1, rowwise=1),
                 "h3_lin2": lambda: ops.gemm_h3(X["a1"], ra1, W2, D, H, H, 0, EPI_BIAS, bias=b2,
                                                rowwise=1),
                 # the step's h3 forward products (row-scaled A)
                 "h3_lin1": lambda: ops.gemm_h3(X["agg"], ragg, W0, H, D, D, 0, EPI_BIAS_RELU,
                                                bias=b0, rowwise=1, bits_out=bits),
                 "w6h_dW2": lambda: ops.linear_wgrad_h3(X["dz"], smax["dz"], X["a1"], smax["a1"],
                                                        Wg2, bg2),
                 "w6h_dW1": lambda: ops.linear_wgrad_h3(X["dz1"], smax["dz1"], X["agg"],
                                                        smax["agg"], Wg0, bg0),
                 "w6_dW2": lambda: ops.linear_bwd(X["dz"], X["a1"], W2, need_x=False),
                 "w6_dW1": lambda: ops.linear_bwd(X["dz1"], X["agg"], W0, need_x=False)}
        fn = cases[case]
    if "--time" in sys.argv:  # median of 5 event-timed runs of `reps` calls
        import statistics
        for _ in range(3):
            fn()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / reps)
        print(f"{case} {statistics.median(ts):.2f} us/call")
        return
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    print("done", case, reps)


if __name__ == "__main__":
    main()
