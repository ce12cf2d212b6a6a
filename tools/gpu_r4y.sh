# usage (GPU box): bash tools/gpu_r4y.sh <tag>: K-Means GPU tests, config 5 bench, headline bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r4y}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_kmeans_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/pytest_$T.log; fatal $rc pytest
timeout -k 10 600 python bench.py --config kmeans_bf16 --cpu-rows 0 --no-estimator --skip-unpruned > gpurun_out/bench_cfg5_$T.json 2> gpurun_out/bench_cfg5_$T.err
rc=$?; echo cfg5_rc=$rc; fatal $rc cfg5
timeout -k 10 300 python bench.py --cpu-rows 0 --no-estimator > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; echo bench_rc=$rc; fatal $rc bench
echo done
