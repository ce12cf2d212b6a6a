#!/bin/bash
# ALS solve timing ablations (OAP_ALS_ABLATE bits, kernels/als.hip): kernel trace per setting.
#   bash tools/als_ablate.sh TAG "0 1 2 4 8"
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$1
shift
cd /tmp && export TMPDIR=/tmp
for b in $1; do
  OAP_ALS_ABLATE=$b timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv \
    -d $R/gpurun_out/alsab_${T}_$b -o run -- python3 $R/benchmarks/bench_als.py \
    --ratings 20000000 --users 1000000 --items 100000 --iters 2 \
    > $R/gpurun_out/alsab_${T}_$b.log 2>&1 || { echo "ablate $b failed rc=$?"; exit 1; }
  echo "ablate=$b"
  python3 $R/tools/trace_summary.py $R/gpurun_out/alsab_${T}_$b 100 | grep als_solve
done
