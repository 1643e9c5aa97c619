#!/bin/bash
# builds benchmarks/probe/libprobe*.so (measurement probes, not the library):
# the eigensolver stamp probe at several prefetch distances (A/B)
cd "$(dirname "$0")" || exit 1
for v in "4 4" "16 8"; do
  set -- $v
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -DSLW_STURM_PF=$1 -DSLW_TWIST_PF=$2 \
    -I ../../libskylark_amd/_native/include -o libprobe_s$1_t$2.so eig_stamps.hip || exit 1
done
