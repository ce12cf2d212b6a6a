#!/bin/bash
# A/B of the headline with and without bound pruning in separate processes (order effects out)
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
A="--no-separable-extra --no-estimator --skip-unpruned --skip-fit"
for rep in 1 2; do
  for mode in prune noprune; do
    extra=""; [ $mode = noprune ] && extra="--no-prune"
    timeout -k 10 200 python bench.py $A $extra > gpurun_out/ab_${mode}_$rep.json 2>/dev/null || exit 1
    python -c "import json; r=json.load(open('gpurun_out/ab_${mode}_$rep.json')); print('$mode', $rep, round(r['ms_per_step'],3), r['extra']['pruned_frac'])"
  done
done
