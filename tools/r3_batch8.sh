#!/bin/bash
# A/B: in-step w6 kernel time, compiler schedule (in-tree) vs interleaved reads (tools/ab/lib_w6i.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ]; }
rm -rf gpurun_out/pa gpurun_out/pb
step pa 400 rocprofv3 --kernel-trace --stats -d gpurun_out/pa -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing &&
MOLCLR_LIB=tools/ab/lib_w6i.so step pb 400 rocprofv3 --kernel-trace --stats -d gpurun_out/pb -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing &&
step ba 300 python bench.py --no-cpu-baseline --no-kernel-timing &&
MOLCLR_LIB=tools/ab/lib_w6i.so step bb 300 python bench.py --no-cpu-baseline --no-kernel-timing &&
step ba2 300 python bench.py --no-cpu-baseline --no-kernel-timing &&
MOLCLR_LIB=tools/ab/lib_w6i.so step bb2 300 python bench.py --no-cpu-baseline --no-kernel-timing
for f in ba bb ba2 bb2; do echo $f; grep -o '"value": [0-9.]*' gpurun_out/$f.log; done
