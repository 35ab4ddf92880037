#!/bin/bash
# Memory-side PMC passes over one GEMM shape (tools/gemm_one.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
IMPL=${IMPL:-bp5}; CASE=${CASE:-lin1}
out=gpurun_out/gpmc2_${IMPL}_${CASE}
rm -rf "$out"; mkdir -p "$out"
n=0
for P in "FETCH_SIZE TCC_HIT_sum" "TCC_MISS_sum WRITE_SIZE" "SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_SALU SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_SMEM"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex gemm -d "$out/p$n" -o run --output-format csv -- python tools/gemm_one.py $IMPL $CASE 10 > "$out/p$n.log" 2>&1 || { echo "pass $n failed"; tail -5 "$out/p$n.log"; exit 1; }
done
python tools/pmc_summary.py "$out"
