# usage (GPU box): bash tools/gpu_r4fc.sh <tag>: K-Means GPU tests + headline bench + shard proxy
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r4fc}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_kmeans_gpu.py tests/test_device_comm_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/pytest_$T.log; fatal $rc pytest
timeout -k 10 300 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; echo bench_rc=$rc; fatal $rc bench
timeout -k 10 300 python bench.py --rows 12500000 --force-rccl --cpu-rows 0 --no-estimator --no-separable-extra > gpurun_out/shard_${T}_n8.json 2> gpurun_out/shard_${T}_n8.err
rc=$?; echo shard_rc=$rc; fatal $rc shard
echo done
