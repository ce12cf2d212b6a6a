# usage (GPU box): bash tools/gpu_round_end.sh <tag>: full GPU suite, smoke(), headline bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-end}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2: stopping"; exit $1;; esac; }
timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/pytest_gpu_$T.log; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$T.txt 2>&1
rc=$?; echo smoke_rc=$rc; tail -1 gpurun_out/smoke_$T.txt; fatal $rc smoke
timeout -k 10 300 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; echo bench_rc=$rc; fatal $rc bench
echo done
