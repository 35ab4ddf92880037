#!/bin/bash
# round-3 batch 2: bf16 ReLU bits + bias preload (c5), q6 epilogue preloads (c2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 "gpurun_out/$name.log"; [ $rc -le 1 ]; }
step bf16t 600 python -m pytest tests/test_gpu_bf16.py -m gpu -q -x --maxfail=5 -rf --timeout 300 --timeout-method thread &&
step kernt 600 python -m pytest tests/test_gpu_kernels.py -m gpu -q --maxfail=20 -rf --timeout 300 --timeout-method thread -k "gemm or q6 or h3 or bplanes" &&
step q6exp2 240 python tools/q6_exp.py &&
step bf16exp2 240 python tools/gemm_bf16_bench.py &&
step bench5 400 python bench.py --no-cpu-baseline --config c5 &&
step bench2 400 python bench.py --no-cpu-baseline &&
step spread2 400 env MOLCLR_Q6_GROUPS=2 python tools/order_spread.py gin gpurun_out/order_spread_gin_kg2.json
