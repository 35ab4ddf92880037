#!/bin/bash
# round-3 measurement batch: GEMM epilogue/K split, bf16 epilogue shapes, cold
# scatter-add (timing, rocprofv3, PMC), molecule-order error spread
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 "gpurun_out/$name.log"; [ $rc -eq 0 ]; }
step q6exp_old 240 env MOLCLR_LIB=tools/ab/lib_old.so python tools/q6_exp.py &&
step q6exp 240 python tools/q6_exp.py &&
step bf16exp 240 python tools/gemm_bf16_bench.py &&
step cold 240 python tools/scatter_cold.py 16 20 cold &&
step warm 240 python tools/scatter_cold.py 16 20 warm &&
rm -rf gpurun_out/coldprof gpurun_out/coldfetch gpurun_out/coldwrite &&
step coldprof 240 rocprofv3 --kernel-trace --stats -d gpurun_out/coldprof -o run --output-format csv -- python tools/scatter_cold.py 16 20 cold &&
step coldfetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_gine_agg_fwd -d gpurun_out/coldfetch -o run --output-format csv -- python tools/scatter_cold.py 16 5 cold &&
step coldwrite 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_gine_agg_fwd -d gpurun_out/coldwrite -o run --output-format csv -- python tools/scatter_cold.py 16 5 cold &&
step spread 400 python tools/order_spread.py gin gpurun_out/order_spread_gin.json
