#!/bin/bash
# w6 with the fragment reads of group g + 2 interleaved with group g's MFMAs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ]; }
step w6t 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x --timeout 300 --timeout-method thread -k "wgrad or colsum or gemm_f32" &&
step h3b 300 python tools/h3_bench.py &&
step b7 300 python bench.py --no-cpu-baseline &&
step b7_5 300 python bench.py --no-cpu-baseline --config c5
tail -3 gpurun_out/w6t.log; grep -v amdgpu.ids gpurun_out/h3b.log
for f in b7 b7_5; do grep -o '"value": [0-9.]*' gpurun_out/$f.log; done
