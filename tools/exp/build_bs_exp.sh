#!/bin/bash
# Builds the B-stationary GEMM experiment library (not shipped; see bs_exp.hip).
set -e
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I../../include \
  -o libbs_exp.so bs_exp.hip
