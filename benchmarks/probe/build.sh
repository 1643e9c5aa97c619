#!/bin/bash
# builds benchmarks/probe/libprobe.so (measurement probes, not the library)
cd "$(dirname "$0")" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC \
  -I ../../libskylark_amd/_native/include -o libprobe.so eig_stamps.hip
