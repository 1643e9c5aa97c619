#!/bin/bash
# FJLT stage-1 ablations (load / FFT / store floors) and UB=32
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
N=benchmarks/native
FS_AB_LIBS=base:$(pwd)/$N/libfs_base.so,ub32:$(pwd)/$N/libfs_ub32.so,nofft:$(pwd)/$N/libfs_nofft.so,nostore:$(pwd)/$N/libfs_nostore.so,noload:$(pwd)/$N/libfs_noload.so,base2:$(pwd)/$N/libfs_base.so \
  timeout -k 10 300 python benchmarks/fjlt_stage1_ab.py > $OUT/fs1_ab.log 2>&1
rc=$?; grep '^{' $OUT/fs1_ab.log; [ $rc -ne 0 ] && tail -20 $OUT/fs1_ab.log; exit $rc
