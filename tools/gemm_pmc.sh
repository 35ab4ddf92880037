#!/bin/bash
# PMC passes over one GEMM shape (tools/gemm_one.py), one rocprofv3 run per pass.
#   IMPL=1 CASE=lin1 bash tools/gemm_pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
IMPL=${IMPL:-1}; CASE=${CASE:-lin1}
out=gpurun_out/gpmc_${IMPL}_${CASE}
rm -rf "$out"; mkdir -p "$out"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS"
n=0
for P in "$P1" "$P2"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex gemm -d "$out/p$n" -o run --output-format csv -- python tools/gemm_one.py $IMPL $CASE 10 > "$out/p$n.log" 2>&1 || { echo "pass $n failed"; tail -5 "$out/p$n.log"; exit 1; }
done
python tools/pmc_summary.py "$out"
