#!/bin/bash
# one GPU round: NT-Xent checks, side-stream checks + A/B, h3 GEMM kernel tests, c2 profile
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 120 ./tools/exp/hsplit_check > gpurun_out/hsplit.log 2>&1; rc=$?; cat gpurun_out/hsplit.log; [ $rc -ne 0 ] && exit $rc
./tools/r5_ntx.sh || exit $?
./tools/r5_side.sh || exit $?
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread \
  tests/test_gpu_kernels.py -k "h3 or gemm or wgrad" > gpurun_out/h3_tests.log 2>&1
rc=$?; tail -2 gpurun_out/h3_tests.log; grep "^E " gpurun_out/h3_tests.log | head -5
[ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing > gpurun_out/prof.log 2>&1
rc=$?; python tools/prof_summary.py gpurun_out/prof gpurun_out/prof.md 25 > /dev/null
exit $rc
