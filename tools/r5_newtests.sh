#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
  tests/test_gpu_models.py tests/test_gpu_dp.py tests/test_gpu_graph_step.py \
  "tests/test_gpu_kernels.py::test_linear_wgrad_h3" > gpurun_out/newtests.log 2>&1
rc=$?; tail -3 gpurun_out/newtests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --dp --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_dp.log 2>&1
rc=$?; tail -1 gpurun_out/bench_dp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['captures'], d['ranks'])"
exit $rc
