#!/bin/bash
# one GPU call: small-LA phase stamps, small-LA / CG / C-ABI GPU tests, the engine probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python benchmarks/core_stamps.py > gpurun_out/core_stamps.log 2>&1 || { echo "core_stamps rc=$?"; tail -20 gpurun_out/core_stamps.log; exit 1; }
cat gpurun_out/core_stamps.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rsvd_core.py tests/test_gpu_krylov.py tests/test_capi.py -m gpu > gpurun_out/step_gpu.log 2>&1 || { echo "tests rc=$?"; grep -E "PASS|FAIL|Error|error" gpurun_out/step_gpu.log | tail -30; tail -30 gpurun_out/step_gpu.log; exit 1; }
tail -3 gpurun_out/step_gpu.log
timeout -k 10 200 python benchmarks/engine_probe.py > gpurun_out/eng.log 2>&1 || { echo "probe rc=$?"; tail -20 gpurun_out/eng.log; exit 1; }
grep -v '^{"k"' gpurun_out/eng.log | tail -8
