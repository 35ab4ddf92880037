#!/bin/bash
# PMC passes over one GEMM shape (tools/gemm_case.py), one rocprofv3 run per pass.
#   CASE=qb_lin2 VARIANT=1 bash tools/gemm_pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CASE=${CASE:-qb_lin2}; VARIANT=${VARIANT:-0}
out=gpurun_out/gpmc_${CASE}_${VARIANT}
rm -rf "$out"; mkdir -p "$out"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS"
P3="FETCH_SIZE TCC_HIT_sum"
n=0
for P in "$P1" "$P2" "$P3"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "gemm|wgrad" -d "$out/p$n" -o run --output-format csv -- python tools/gemm_case.py $CASE 10 $VARIANT > "$out/p$n.log" 2>&1 || { echo "pass $n failed"; tail -5 "$out/p$n.log"; exit 1; }
done
python tools/pmc_summary.py "$out"
