# usage (GPU box): bash tools/gpu_als_prof.sh <tag>: ALS 1B kernel trace (stats)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-alsprof}
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$T -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_als.py --iters 2 --cpu-ratings 0 > $GRAFT_REPO_ROOT/gpurun_out/$T.log 2>&1)
rc=$?; echo prof_rc=$rc
