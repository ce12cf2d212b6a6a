#!/bin/bash
# usage (GPU box): tools/pmc_pca.sh <tag>: PMC passes over the exact PCA SYRK (oap_pca_syrk_f64)
# at 10M x 1000 (kernel trace + counters only; no sys/runtime traces)
set -u
R=$GRAFT_REPO_ROOT; T=${1:-pmcpca}
cd /tmp && export TMPDIR=/tmp
run() {
  local P=$1; shift
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T}_$P -o run \
    --kernel-include-regex syrk_f64 --pmc "$@" -- python3 $R/benchmarks/bench_pca.py --reps 1 \
    --cpu-rows 0 --precision exact > $R/gpurun_out/${T}_$P.log 2>&1
  local rc=$?; echo "pmc_${P}_rc=$rc"; return $rc
}
run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE && \
run b SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE && \
run c SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAVE_CYCLES GRBM_GUI_ACTIVE && \
run d TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE
