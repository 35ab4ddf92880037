#!/bin/bash
# w6 (weight gradient) main-loop ablations
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ]; }
step w6abl 300 python tools/w6_abl.py
grep -v amdgpu.ids gpurun_out/w6abl.log
