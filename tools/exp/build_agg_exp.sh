#!/bin/bash
# Builds the scatter-add experiment library (not shipped; see agg_exp.hip).
set -e
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I../../include \
  -o libagg_exp.so agg_exp.hip
