#!/bin/bash
# usage (GPU box): tools/als_ablate.sh <tag> <ablate>...  — one rocprofv3 kernel-stats run of
# benchmarks/bench_als.py per OAP_ALS_ABLATE value (timing ablations, results are not factors)
set -u
R=$GRAFT_REPO_ROOT; T=$1; shift
mkdir -p $R/gpurun_out
for ab in "$@"; do
  (cd /tmp && export TMPDIR=/tmp && OAP_ALS_ABLATE=$ab timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/alsab_${T}_$ab -o run -- python3 $R/benchmarks/bench_als.py --iters 1 ${ALS_ARGS:-} > $R/gpurun_out/alsab_${T}_$ab.log 2>&1)
  rc=$?; echo "ablate=$ab rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
  python3 - "$R/gpurun_out/alsab_${T}_$ab" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)
for r in list(csv.DictReader(open(f[0])))[:10]:
    print(f"  {r['Name'][:70]:70s} {int(r['Calls']):4d} {int(r['TotalDurationNs'])/1e6:9.2f} ms")
PY
done
