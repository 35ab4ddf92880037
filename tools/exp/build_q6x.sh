#!/bin/bash
# q6 main-loop variant library (tools/q6x.py); not part of the product build
set -e
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -I ../../include q6x.hip -o libq6x.so
