#!/bin/bash
# q6 ablation round 6: 8-wave blocks sharing one B stage
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ]; }
step q6abl6 300 python tools/q6_abl.py
grep -v amdgpu.ids gpurun_out/q6abl6.log
