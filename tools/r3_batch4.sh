#!/bin/bash
# q6 B staging by LDS-DMA vs registers: ablation harness, GEMM shapes, parity
# tests, c2 bench (tools/ab/lib_reg.so = register staging, in-tree = DMA)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ]; }
step q6abl4 300 python tools/q6_abl.py &&
step q6x_reg 240 env MOLCLR_LIB=tools/ab/lib_reg.so python tools/q6_exp.py &&
step q6x_dma 240 python tools/q6_exp.py &&
step kern_dma 600 python -m pytest tests/test_gpu_kernels.py -m gpu -q --maxfail=20 -rf --timeout 300 --timeout-method thread -k "gemm or q6 or h3 or bplanes or linear" &&
step b_reg 300 env MOLCLR_LIB=tools/ab/lib_reg.so python bench.py --no-cpu-baseline &&
step b_dma 300 python bench.py --no-cpu-baseline &&
step b_reg2 300 env MOLCLR_LIB=tools/ab/lib_reg.so python bench.py --no-cpu-baseline --no-kernel-timing &&
step b_dma2 300 python bench.py --no-cpu-baseline --no-kernel-timing
for f in q6abl4 q6x_reg q6x_dma; do grep -v amdgpu.ids gpurun_out/$f.log | head -24; done
tail -3 gpurun_out/kern_dma.log
for f in b_reg b_dma b_reg2 b_dma2; do grep -o '"value": [0-9.]*' gpurun_out/$f.log; done
