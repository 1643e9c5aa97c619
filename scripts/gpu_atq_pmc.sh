set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for b in 1 0; do
  SL_ATQ_BF16=$b timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_INSTS_VALU -d $R/gpurun_out/atq_pmc_$b -o run --output-format csv -- python3 $R/benchmarks/probe/atq_time.py one > $R/gpurun_out/atq_pmc_$b.log 2>&1 || exit 1
done
