#!/bin/bash
# usage (on the GPU box, after the build): tools/pmc_lean.sh <tag> [sigma] [variant] [ablation]
# PMC passes over the lean K-Means pass (kernel trace + counters only — no sys/runtime traces).
set -u
R=$GRAFT_REPO_ROOT; T=${1:-pmc}; S=${2:-8}; V=${3:-0}; A=${4:-0}
cd /tmp && export TMPDIR=/tmp
run() {  # $1 = pass name, rest = counters
  local P=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T}_$P -o run \
    --pmc "$@" -- python3 $R/tools/kmeans_lean_probe.py 20000000 $S 3 $V $A \
    > $R/gpurun_out/${T}_$P.log 2>&1
  local rc=$?; echo "pmc_${P}_rc=$rc"; return $rc
}
[ -n "${ONLY_B:-}" ] || run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE && \
run b SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE && \
run c SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
