#!/bin/bash
# PMC counters of the fused randSVD pass (inter: final 0; last pass: final 1,
# Y + fp64 Gram), one rocprofv3 run per counter group (hardware slot limits:
# <= 8 SQ, <= 4 TCC, <= 2 GRBM), kernel trace only alongside; CSVs under
# gpurun_out/pmc5/.  Summary: scripts/pmc_summary.py.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc5
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for SET in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU" \
           "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT" \
           "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  for F in 0 1; do
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $SET --output-format csv -d $OUT/f${F}_g$i -o run -- \
      python3 $R/benchmarks/bench_pass.py --variants 0 --finals $F --reps 6 > $OUT/f${F}_g$i.log 2>&1 \
      || { echo "pmc set $i final $F failed"; tail -5 $OUT/f${F}_g$i.log; exit 1; }
  done
done
echo pmc done
