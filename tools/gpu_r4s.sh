# usage (GPU box): bash tools/gpu_r4s.sh <tag>: adaptive fused scan: tests, bench A/B, shard n8, trace
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r4s}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_kmeans_gpu.py -v --timeout 200 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/pytest_$T.log; fatal $rc pytest
timeout -k 10 300 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; echo bench_rc=$rc; fatal $rc bench
OAP_KMEANS_SCAN_ADAPT=0 timeout -k 10 300 python bench.py --cpu-rows 0 --no-estimator > gpurun_out/bench_${T}_noadapt.json 2> gpurun_out/bench_${T}_noadapt.err
rc=$?; echo bench_na_rc=$rc; fatal $rc bench_na
timeout -k 10 300 python bench.py --rows 12500000 --force-rccl --cpu-rows 0 --no-estimator --no-separable-extra > gpurun_out/shard_${T}_n8.json 2> gpurun_out/shard_${T}_n8.err
rc=$?; echo shard_rc=$rc; fatal $rc shard
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/trace_bench_$T -o run -- python3 $GRAFT_REPO_ROOT/bench.py --warmup 1 --skip-fit --skip-unpruned --no-separable-extra --no-estimator --cpu-rows 0 > $GRAFT_REPO_ROOT/gpurun_out/trace_bench_$T.log 2>&1)
rc=$?; echo trace_rc=$rc; fatal $rc trace
echo done
