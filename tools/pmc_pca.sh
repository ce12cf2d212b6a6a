#!/bin/bash
# usage (on the GPU box, after the build): tools/pmc_pca.sh <tag>
# Kernel trace + one PMC pass over the PCA SYRK kernel (2 reps of the 10M x 1000 benchmark).
set -u
R=$GRAFT_REPO_ROOT; T=${1:-pmcpca}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T}a -o run \
  --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES \
  -- python3 $R/benchmarks/bench_pca.py --reps 1 > $R/gpurun_out/${T}a.log 2>&1
rc=$?; echo pmc_a_rc=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T}b -o run \
  --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
  -- python3 $R/benchmarks/bench_pca.py --reps 1 > $R/gpurun_out/${T}b.log 2>&1
rc=$?; echo pmc_b_rc=$rc; exit $rc
