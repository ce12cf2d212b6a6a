#!/bin/bash
# HBM traffic of the PCA SYRK (one PMC pass: TCC FETCH_SIZE + SQ_WAVES)
set -u
R=$GRAFT_REPO_ROOT; T=${1:-pmcpcamem}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T} -o run \
  --pmc FETCH_SIZE SQ_WAVES GRBM_GUI_ACTIVE \
  -- python3 $R/benchmarks/bench_pca.py --reps 1 > $R/gpurun_out/${T}.log 2>&1
rc=$?; echo pmc_rc=$rc; exit $rc
