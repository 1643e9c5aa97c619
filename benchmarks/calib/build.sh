#!/bin/bash
# builds benchmarks/calib/libcalib.so (calibration kernels, not the library)
cd "$(dirname "$0")" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o libcalib.so gather.hip
