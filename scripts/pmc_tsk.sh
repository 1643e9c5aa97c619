#!/bin/bash
# PMC counter passes over the fused pass (inter variant: flags 3, no Gram),
# one rocprofv3 run per counter group (hardware slot limits), CSVs under
# gpurun_out/pmc_tsk/<group>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU" \
           "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/pmc_tsk${PMC_TAG:-}/g$i" -o pmc -- python3 "$R/benchmarks/fused_once.py" "$@" > "$R/gpurun_out/pmc_tsk${PMC_TAG:-}_g$i.log" 2>&1 || exit 1
done
