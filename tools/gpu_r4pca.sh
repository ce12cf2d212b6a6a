# usage (GPU box): bash tools/gpu_r4pca.sh <tag>: PCA GPU tests + the 10M x 1000 PCA bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r4pca}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_pca_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/pytest_$T.log; fatal $rc pytest
timeout -k 10 300 python benchmarks/bench_pca.py --cpu-rows 0 --precision exact > gpurun_out/bench_pca_$T.json 2> gpurun_out/bench_pca_$T.err
rc=$?; echo bench_rc=$rc; fatal $rc bench
echo done
