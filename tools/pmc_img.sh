#!/bin/bash
# usage (on the GPU box, after the build): tools/pmc_img.sh <tag> [cfg list] [rows]
# PMC passes over the steady-state image pass (tools/kmeans_img_probe.py): kernel trace +
# counters only (no sys/runtime traces).  Summaries: tools/pmc_summary.py --kernel lean_img.
set -u
R=$GRAFT_REPO_ROOT; T=${1:-pmcimg}; C=${2:--1}; N=${3:-20000000}
cd /tmp && export TMPDIR=/tmp PROBE_FALLBACK=0
run() {  # $1 = pass name, rest = counters
  local P=$1; shift
  timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T}_$P -o run \
    --pmc "$@" -- python3 $R/tools/kmeans_img_probe.py $N 8 2 $C \
    > $R/gpurun_out/${T}_$P.log 2>&1
  local rc=$?; echo "pmc_${P}_rc=$rc"; return $rc
}
run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE && \
run b SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE && \
run c SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
