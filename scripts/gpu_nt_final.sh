set -o pipefail
VAR=SL_PASS_NT_FINAL VALS="0 1" PAT=k_xm_pipe bash scripts/ab_env_prof.sh > gpurun_out/nt_final_xm.log 2>&1 || exit 1
VAR=SL_PASS_NT_FINAL VALS="0 1" PAT=k_rsvd_pass5 bash scripts/ab_env_prof.sh > gpurun_out/nt_final_pass.log 2>&1
