#!/bin/bash
# usage (on the GPU box): tools/pmc_pca.sh <tag> — PMC passes over the PCA fit (2M x 1000, or
# PCA_PMC_ARGS; kernel trace + counters only, no sys/runtime traces).
set -u
R=$GRAFT_REPO_ROOT; T=${1:-pmcpca}
cd /tmp && export TMPDIR=/tmp
run() {
  local P=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T}_$P -o run \
    --pmc "$@" -- python3 $R/benchmarks/bench_pca.py ${PCA_PMC_ARGS:---rows 2000000} \
    --reps 1 > $R/gpurun_out/${T}_$P.log 2>&1
  local rc=$?; echo "pmc_${P}_rc=$rc"; return $rc
}
run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE && \
run b SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE && \
run c SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
