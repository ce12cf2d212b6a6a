# usage (GPU box): bash tools/gpu_round_end2.sh <tag>: full GPU suite, smoke(), headline bench,
# 12.5M-row shard proxy, PCA exact bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-end}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2: stopping"; exit $1;; esac; }
timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/pytest_gpu_$T.log; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$T.txt 2>&1
rc=$?; echo smoke_rc=$rc; tail -1 gpurun_out/smoke_$T.txt; fatal $rc smoke
timeout -k 10 300 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; echo bench_rc=$rc; fatal $rc bench
timeout -k 10 300 python bench.py --rows 12500000 --force-rccl --cpu-rows 0 --no-estimator --no-separable-extra > gpurun_out/shard_${T}_n8.json 2> gpurun_out/shard_${T}_n8.err
rc=$?; echo shard_rc=$rc; fatal $rc shard
timeout -k 10 300 python benchmarks/bench_pca.py --cpu-rows 0 --precision exact > gpurun_out/bench_pca_$T.json 2> gpurun_out/bench_pca_$T.err
rc=$?; echo pca_rc=$rc; fatal $rc pca
echo done
