# usage (GPU box): bash tools/gpu_r4g.sh <tag>; K-Means fused row scan + recommend kernel
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r4g}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_recommend_gpu.py tests/test_kmeans_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/pytest_$T.log; fatal $rc pytest
timeout -k 10 300 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; echo bench_rc=$rc; fatal $rc bench
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/trace_bench_$T -o run -- python3 $GRAFT_REPO_ROOT/bench.py --warmup 0 --skip-fit --skip-unpruned --no-separable-extra --no-estimator --cpu-rows 0 > $GRAFT_REPO_ROOT/gpurun_out/trace_bench_$T.log 2>&1)
rc=$?; echo trace_rc=$rc; fatal $rc trace
timeout -k 10 300 python benchmarks/bench_recommend.py --users 2000000 --items 500000 > gpurun_out/bench_rec_small_$T.json 2> gpurun_out/bench_rec_small_$T.err
rc=$?; echo rec_small_rc=$rc; fatal $rc rec_small
echo done
