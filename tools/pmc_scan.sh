#!/bin/bash
# usage (GPU box): tools/pmc_scan.sh <tag>: PMC passes over oap_kmeans_lean_img in a short
# headline bench (pruned fit: fused-scan passes; unpruned fit: dense passes)
set -u
R=$GRAFT_REPO_ROOT; T=${1:-pmcscan}
cd /tmp && export TMPDIR=/tmp
run() {
  local P=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T}_$P -o run \
    --kernel-include-regex lean_img --pmc "$@" -- python3 $R/bench.py --steps 8 --warmup 0 \
    --skip-fit --no-separable-extra --no-estimator --cpu-rows 0 \
    > $R/gpurun_out/${T}_$P.log 2>&1
  local rc=$?; echo "pmc_${P}_rc=$rc"; return $rc
}
run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE && \
run b SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE && \
run c SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
