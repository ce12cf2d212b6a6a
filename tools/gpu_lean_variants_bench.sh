#!/bin/bash
# headline bench per lean-kernel workgroup shape (OAP_KMEANS_LEAN_VARIANT), short form
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${1:-lv}; shift
for v in "$@"; do
  OAP_KMEANS_LEAN_VARIANT=$v timeout -k 10 200 python bench.py --no-separable-extra --no-estimator --skip-unpruned --skip-fit > gpurun_out/bench_${T}_v$v.json 2> gpurun_out/bench_${T}_v$v.err
  rc=$?; [ $rc -ne 0 ] && { echo "variant $v rc=$rc"; tail -3 gpurun_out/bench_${T}_v$v.err; exit $rc; }
  python -c "import json,sys; r=json.load(open('gpurun_out/bench_${T}_v$v.json')); print('variant', $v, 'ms_per_step', round(r['ms_per_step'],3), 'assign_ms', round(r['extra']['assign_kernel_ms'],3), r['extra'].get('image_passes'))"
done
