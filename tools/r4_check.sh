#!/bin/bash
# Round-4 GPU check: parity suites first (stop on a crash), then benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name limit cmd...: a test step may fail (rc 1) without stopping the run
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/$name.log"
  [ $rc -le 1 ]
}
T="python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread -rf"
for s in ${STEPS:-kernels models graph bench bench3}; do
  case $s in
    kernels) step kernels 900 $T tests/test_gpu_kernels.py || exit 1 ;;
    models)  step models 900 $T tests/test_gpu_models.py || exit 1 ;;
    graph)   step graph 600 $T tests/test_gpu_graph_step.py tests/test_gpu_dp.py || exit 1 ;;
    rest)    step rest 900 $T tests --deselect tests/test_gpu_kernels.py --deselect tests/test_gpu_models.py || exit 1 ;;
    all)     step all 1100 $T tests || exit 1 ;;
    bench)   step bench 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1 ;;
    bench5)  step bench5 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --config c5 || exit 1 ;;
    bench3)  step bench3 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --config c3 || exit 1 ;;
    prof)    rm -rf gpurun_out/prof; step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing || exit 1 ;;
    prof5)   rm -rf gpurun_out/prof5; step prof5 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run --output-format csv -- python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing || exit 1 ;;
    smoke)   step smoke 300 python __graft_entry__.py smoke || exit 1 ;;
  esac
done
