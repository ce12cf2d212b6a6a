# PMC passes of round 5 (run through gpurun): the ALS low-rank solves at 200M ratings and the
# headline's row-scan image passes
set -u
cd $GRAFT_REPO_ROOT
export PROBE_ARGS="--ratings 200000000 --users 4000000 --items 400000 --iters 2 --cpu-ratings 0"
for p in mem fetch a b; do bash tools/gpu.sh als pmc:../benchmarks/bench_als.py:$p || exit $?; done
export PROBE_ARGS="--warmup 0 --skip-fit --skip-unpruned --no-separable-extra --no-estimator --cpu-rows 0"
for p in mem fetch a b; do bash tools/gpu.sh head pmc:../bench.py:$p || exit $?; done
