#!/bin/bash
# diagnostic build of rsvd_core.hip with phase stamps (benchmarks/core_stamps.py)
set -eu
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc -O3 -fPIC -shared -std=c++17 --offload-arch=gfx950 -DSL_CORE_STAMPS \
  -I libskylark_amd/_native/include libskylark_amd/_native/src/rsvd_core.hip \
  benchmarks/native/stub_err.hip -o benchmarks/native/libcore_stamps.so
