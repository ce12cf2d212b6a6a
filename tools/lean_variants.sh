#!/bin/bash
# lean-pass variants (tools/kmeans_lean_probe.py) at sigma 8: ablation 5 (distance + argmin +
# labels) and 0 (full pass), ms per 100M rows
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in 0 3 5 6 7 8 9 10; do
  timeout -k 10 120 python tools/kmeans_lean_probe.py 30000000 8 6 $v 5,1 >> gpurun_out/lean_variants_$1.jsonl 2>/dev/null
  rc=$?; [ $rc -ne 0 ] && { echo "variant $v rc=$rc"; exit $rc; }
done
cat gpurun_out/lean_variants_$1.jsonl
