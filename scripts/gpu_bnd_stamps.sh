set -o pipefail
mkdir -p gpurun_out
LIB=libskylark_amd/_native/libskylark_hip.so
cp $LIB /tmp/lib_keep.so && cp stamps.so $LIB || exit 1
timeout -k 10 200 python -u benchmarks/probe/bnd_stamps.py > gpurun_out/bnd_stamps.log 2>&1; rc=$?
cp /tmp/lib_keep.so $LIB
exit $rc
