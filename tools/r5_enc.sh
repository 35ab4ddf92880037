#!/bin/bash
# executor vs per-op bit-identity: this tree's library, then the ff83622 one
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T="tests/test_gpu_models.py::test_encoder_executor_matches_per_op_path tests/test_gpu_kernels.py::test_linear_wgrad_h3_pair_matches_two_calls tests/test_gpu_kernels.py::test_fused_adam_matches_torch_adam"
for v in new ff; do
  if [ $v = ff ]; then export MOLCLR_LIB=$PWD/tools/exp/libmolclr_ff.so; fi
  timeout -k 10 200 python -u -m pytest -q -m gpu --timeout 100 --timeout-method thread $T > gpurun_out/enc_$v.log 2>&1
  rc=$?; echo "$v rc=$rc $(tail -1 gpurun_out/enc_$v.log)"; grep "^FAILED" gpurun_out/enc_$v.log | head -4
  [ $rc -gt 1 ] && exit $rc
done
exit 0
