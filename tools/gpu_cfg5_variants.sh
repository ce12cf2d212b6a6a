#!/bin/bash
# config-5 shape (k=1000, d=100 bf16) at a reduced row count per lean-kernel workgroup shape
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${1:-c5v}; ROWS=${ROWS:-200000000}; shift
for v in "$@"; do
  OAP_KMEANS_LEAN_VARIANT=$v timeout -k 10 300 python bench.py --config kmeans_bf16 --rows $ROWS --steps 6 --warmup 1 --no-separable-extra --no-estimator --skip-unpruned --skip-fit > gpurun_out/bench_${T}_v$v.json 2> gpurun_out/bench_${T}_v$v.err
  rc=$?; [ $rc -ne 0 ] && { echo "variant $v rc=$rc"; tail -3 gpurun_out/bench_${T}_v$v.err; exit $rc; }
  python -c "import json; r=json.load(open('gpurun_out/bench_${T}_v$v.json')); print('variant', $v, 'ms_per_step', round(r['ms_per_step'],2), r['extra']['distance_path'])"
done
