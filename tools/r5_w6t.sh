#!/bin/bash
# transposed-orientation h3 weight gradients: kernel + model parity, then c2 bench + profile
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_graph_step.py tests/test_gpu_dp.py \
  > gpurun_out/w6t.log 2>&1
rc=$?; tail -2 gpurun_out/w6t.log; grep "^E " gpurun_out/w6t.log | head -6
[ $rc -ne 0 ] && exit $rc
./tools/r5_ab.sh
