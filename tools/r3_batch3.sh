#!/bin/bash
# q6 K groups: accuracy (tools/order_spread.py) vs speed at c2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' "gpurun_out/$name.log"; [ $rc -eq 0 ]; }
timeout -k 10 200 python tools/q6_abl.py > gpurun_out/q6abl.log 2>&1; echo "q6abl rc=$?"; cat gpurun_out/q6abl.log | grep -v amdgpu.ids
step kgdef 300 python bench.py --no-cpu-baseline --no-kernel-timing &&
step kg2 300 env MOLCLR_Q6_GROUPS=2 python bench.py --no-cpu-baseline --no-kernel-timing &&
step kgdef_b 300 python bench.py --no-cpu-baseline --no-kernel-timing &&
step kg2_b 300 env MOLCLR_Q6_GROUPS=2 python bench.py --no-cpu-baseline --no-kernel-timing &&
step kg2_c3 300 env MOLCLR_Q6_GROUPS=2 python bench.py --no-cpu-baseline --no-kernel-timing --config c3 &&
step kgdef_c3 300 python bench.py --no-cpu-baseline --no-kernel-timing --config c3
