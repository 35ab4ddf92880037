#!/bin/bash
# Round-5 final GPU pass: parity suite, smoke, bench lines, rocprof summaries,
# a PMC pass on the h3 forward GEMM, trainer bench.  Each step under its own
# time limit; stops at the first crash (a test failure, rc 1, does not stop it).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-240
  [ $rc -le 1 ]
}
for s in ${STEPS:-tests smoke bench prof bench5 bench3 benchdp prof5 pmcagg pmc pmcw6 tbench}; do
  case $s in
    tests)   step tests 600 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests -p no:cacheprovider -rf || exit 1 ;;
    smoke)   step smoke 200 python __graft_entry__.py smoke || exit 1 ;;
    bench)   step bench 400 python bench.py || exit 1 ;;
    bench5)  step bench5 300 python bench.py --config c5 --no-cpu-baseline || exit 1 ;;
    bench3)  step bench3 300 python bench.py --config c3 --no-cpu-baseline || exit 1 ;;
    benchdp) step benchdp 300 python bench.py --dp --no-cpu-baseline || exit 1 ;;
    prof)    rm -rf gpurun_out/prof; step prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing || exit 1
             python tools/prof_summary.py gpurun_out/prof gpurun_out/prof.md 25 > /dev/null ;;
    prof5)   rm -rf gpurun_out/prof5; step prof5 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run --output-format csv -- python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing || exit 1
             python tools/prof_summary.py gpurun_out/prof5 gpurun_out/prof5.md 25 > /dev/null ;;
    pmc)     CASE=h3_lin1 VARIANT=0 step gpmc_h3_lin1 400 bash tools/gemm_pmc.sh || exit 1 ;;
    pmcw6)   CASE=w6h_dW1 VARIANT=0 step gpmc_w6h_dW1 400 bash tools/gemm_pmc.sh || exit 1 ;;
    pmcagg)  # HBM traffic of the scatter-add in the step: FETCH_SIZE and WRITE_SIZE in separate passes
             for c in FETCH_SIZE WRITE_SIZE; do
               rm -rf gpurun_out/pmc_$c
               step pmc_$c 120 rocprofv3 --pmc $c --kernel-include-regex k_gine_agg_fwd -d gpurun_out/pmc_$c -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-hip-graph || exit 1
             done
             python tools/pmc_traffic.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE gpurun_out/r5_pmc_gine_agg_c2_pair.json ;;
    tbench)  step tbench_c2_node 400 python -u tools/trainer_bench.py --config c2 --aug node || exit 1 ;;
  esac
done
exit 0
