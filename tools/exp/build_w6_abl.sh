#!/bin/bash
# w6 ablation experiment library (tools/w6_abl.py); not part of the product build
set -e
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -I ../../include w6_abl.hip -o libw6_abl.so
