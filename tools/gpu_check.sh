#!/bin/bash
# GPU-box check: per-step time limits; stop on anything worse than a test failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  return $rc
}
steps="${STEPS:-kernels models bench}"
for s in $steps; do
  case $s in
    kernels) run kernels 900 python -m pytest tests/test_gpu_kernels.py -m gpu -q --maxfail=200 -rf --timeout 300 --timeout-method thread; rc=$? ; [ $rc -le 1 ] || exit $rc ;;
    models)  MOLCLR_RECORD_ERRS=gpurun_out/errs run models 900 python -m pytest tests/test_gpu_models.py -m gpu -q --maxfail=200 -rf --timeout 300 --timeout-method thread; rc=$? ; [ $rc -le 1 ] || exit $rc ;;
    dp)      run dp 600 python -m pytest tests/test_gpu_dp.py -m gpu -q --maxfail=200 -rf --timeout 300 --timeout-method thread; rc=$? ; [ $rc -le 1 ] || exit $rc ;;
    rest)    run rest 900 python -m pytest tests -m gpu -q --maxfail=200 -rf --timeout 300 --timeout-method thread --deselect tests/test_gpu_kernels.py --deselect tests/test_gpu_models.py --deselect tests/test_gpu_dp.py; rc=$? ; [ $rc -le 1 ] || exit $rc ;;
    pmc)     export TMPDIR=/tmp; rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
             run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_gine_agg_fwd -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing; rc=$?; [ $rc -eq 0 ] || exit $rc
             run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_gine_agg_fwd -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    pmc5)    export TMPDIR=/tmp; rm -rf gpurun_out/pmc5_fetch gpurun_out/pmc5_write
             run pmc5_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_gine_agg_fwd -d gpurun_out/pmc5_fetch -o run --output-format csv -- python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing; rc=$?; [ $rc -eq 0 ] || exit $rc
             run pmc5_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_gine_agg_fwd -d gpurun_out/pmc5_write -o run --output-format csv -- python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    gemm)    run gemm 300 python tools/gemm_bench.py 30556; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    ntx)     run ntx 300 python tools/ntxent_scale.py; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    ntxprof) export TMPDIR=/tmp; rm -rf gpurun_out/ntxprof
             run ntxprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ntxprof -o run --output-format csv -- python tools/ntxent_scale.py; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    gemmbf)  run gemmbf 300 python tools/gemm_bf16_bench.py; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    gpmc)    for c in ${PMC_CASES:-qb_lin2:1}; do
               CASE=${c%%:*} VARIANT=${c##*:} run "gpmc_${c%%:*}_${c##*:}" 400 bash tools/gemm_pmc.sh; rc=$?; [ $rc -eq 0 ] || exit $rc
             done ;;
    graph)   run graph 600 python -m pytest tests/test_gpu_graph_step.py -m gpu -q --maxfail=50 -rf --timeout 300 --timeout-method thread; rc=$? ; [ $rc -le 1 ] || exit $rc ;;
    augment) run augment 600 python -m pytest tests/test_gpu_augment.py -m gpu -q --maxfail=50 -rf --timeout 300 --timeout-method thread; rc=$? ; [ $rc -le 1 ] || exit $rc ;;
    trainer) run trainer 600 python -m pytest tests/test_gpu_trainer.py -m gpu -q --maxfail=50 -rf --timeout 300 --timeout-method thread; rc=$? ; [ $rc -le 1 ] || exit $rc ;;
    benche)  run benche 600 python bench.py --no-cpu-baseline --no-hip-graph; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    bench3e) run bench3e 600 python bench.py --no-cpu-baseline --config c3 --no-hip-graph; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    smoke)   run smoke 300 python __graft_entry__.py smoke; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    bench)   run bench 600 python bench.py --no-cpu-baseline; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    bench2)  run bench2 600 python bench.py --no-cpu-baseline --two-pass; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    bf16)    run bf16 900 python -m pytest tests/test_gpu_bf16.py -m gpu -q --maxfail=200 -rf --timeout 300 --timeout-method thread; rc=$? ; [ $rc -le 1 ] || exit $rc ;;
    bench5)  run bench5 600 python bench.py --no-cpu-baseline --config c5; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    bench3)  run bench3 600 python bench.py --no-cpu-baseline --config c3; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    benchfull) run benchfull 900 python bench.py; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    benchd)  run benchd 600 python bench.py --steps 20 --warmup 5; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    benchdp) run benchdp 600 python bench.py --dp --steps 20 --warmup 5 --no-cpu-baseline; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    benchd5) run benchd5 600 python bench.py --steps 20 --warmup 5 --config c5 --no-cpu-baseline; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    benchd3) run benchd3 600 python bench.py --steps 20 --warmup 5 --config c3 --no-cpu-baseline; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    tbench)  for c in ${TB_CASES:-c2:node c2:subgraph c2:mix c3:node}; do
               run "tbench_${c%%:*}_${c##*:}" 600 python -u tools/trainer_bench.py --config ${c%%:*} --aug ${c##*:}; rc=$?; [ $rc -eq 0 ] || exit $rc
             done ;;
    prof5)   export TMPDIR=/tmp; rm -rf gpurun_out/prof5
             run prof5 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run --output-format csv -- python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    prof)    export TMPDIR=/tmp; rm -rf gpurun_out/prof
             run prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
  esac
done
exit 0
