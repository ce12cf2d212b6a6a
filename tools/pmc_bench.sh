#!/bin/bash
# usage (GPU box, after the build): tools/pmc_bench.sh <tag> [rows]
# PMC passes over the headline Lloyd fit (bench.py, delta passes on the operand image), one
# counter group per run, kernel trace + counters only.  Set OAP_KMEANS_REG_PLANE etc. outside.
set -u
R=$GRAFT_REPO_ROOT; T=${1:-pmcb}; N=${2:-20000000}
cd /tmp && export TMPDIR=/tmp
run() {  # $1 = pass name, rest = counters
  local P=$1; shift
  timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T}_$P -o run \
    --pmc "$@" -- python3 $R/bench.py --rows $N --steps 4 --warmup 0 --skip-fit --skip-unpruned \
    --no-separable-extra --no-estimator > $R/gpurun_out/${T}_$P.log 2>&1
  local rc=$?; echo "pmc_${P}_rc=$rc"; return $rc
}
run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE && \
run b SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE && \
run c SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
