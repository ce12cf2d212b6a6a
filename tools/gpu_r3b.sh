#!/bin/bash
# round-3 GPU pass: full GPU suite, headline bench (with the estimator fit), forced-RCCL ALS at
# 1B ratings, and a kernel trace of the forced-RCCL ALS (comm-stream broadcasts vs solves)
set -u
R=$GRAFT_REPO_ROOT; T=${1:-r3b}
cd $R; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -4 gpurun_out/pytest_gpu_$T.log; fatal $rc pytest
timeout -k 10 400 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; echo bench_rc=$rc; cat gpurun_out/bench_$T.json; fatal $rc bench
timeout -k 10 400 python benchmarks/bench_pca.py > gpurun_out/bench_pca_$T.json 2> gpurun_out/bench_pca_$T.err
rc=$?; echo pcabench_rc=$rc; cat gpurun_out/bench_pca_$T.json; fatal $rc pcabench
timeout -k 10 400 python benchmarks/bench_als.py --force-rccl --iters 3 > gpurun_out/bench_als_rccl_$T.json 2> gpurun_out/bench_als_rccl_$T.err
rc=$?; echo alsbench_rc=$rc; cat gpurun_out/bench_als_rccl_$T.json; tail -3 gpurun_out/bench_als_rccl_$T.err; fatal $rc alsbench
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/alsprof_rccl_$T -o run -- python3 $R/benchmarks/bench_als.py --force-rccl --ratings 200000000 --users 4000000 --items 400000 --iters 2 > $R/gpurun_out/alsprof_rccl_$T.log 2>&1)
rc=$?; echo alsprof_rc=$rc; fatal $rc alsprof
