#!/bin/bash
# A/B at c2 and c5: in-tree vs tools/ab/lib_base.so (the previous commit)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ]; }
rm -rf gpurun_out/pa5 gpurun_out/pb5 gpurun_out/pa gpurun_out/pb
step kb 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_graph_step.py tests/test_gpu_models.py -m gpu -q -x --timeout 300 --timeout-method thread &&
step pb 400 rocprofv3 --kernel-trace --stats -d gpurun_out/pb -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing &&
MOLCLR_LIB=tools/ab/lib_base.so step pa 400 rocprofv3 --kernel-trace --stats -d gpurun_out/pa -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing &&
step pb5 400 rocprofv3 --kernel-trace --stats -d gpurun_out/pb5 -o run --output-format csv -- python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing &&
MOLCLR_LIB=tools/ab/lib_base.so step pa5 400 rocprofv3 --kernel-trace --stats -d gpurun_out/pa5 -o run --output-format csv -- python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing &&
step bb 300 python bench.py --no-cpu-baseline --no-kernel-timing &&
MOLCLR_LIB=tools/ab/lib_base.so step ba 300 python bench.py --no-cpu-baseline --no-kernel-timing &&
step bb5 300 python bench.py --config c5 --no-cpu-baseline --no-kernel-timing &&
MOLCLR_LIB=tools/ab/lib_base.so step ba5 300 python bench.py --config c5 --no-cpu-baseline --no-kernel-timing
tail -2 gpurun_out/kb.log
for f in ba bb ba5 bb5; do echo $f; grep -o '"value": [0-9.]*' gpurun_out/$f.log; done
