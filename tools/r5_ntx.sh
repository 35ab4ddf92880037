#!/bin/bash
# NT-Xent / max-slot kernels: their GPU tests, then the c4 rank shard under rocprofv3.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_dp.py -k "ntxent or h3 or absmax or planes or dp" \
  > gpurun_out/ntx_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ntx_tests.log; grep "^E " gpurun_out/ntx_tests.log | head -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/ntxent_c4.py 50 > gpurun_out/ntx_c4.log 2>&1
rc=$?; tail -4 gpurun_out/ntx_c4.log
[ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/ntxprof
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ntxprof -o run --output-format csv -- python tools/ntxent_c4.py 20 > gpurun_out/ntxprof.log 2>&1
rc=$?; python tools/prof_summary.py gpurun_out/ntxprof gpurun_out/ntxprof.md 12 > /dev/null
exit $rc
