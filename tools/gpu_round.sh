#!/bin/bash
# usage: tools/gpu_round.sh <tag> [steps...]  -- on the GPU box: the named steps (default: test
# bench precise prof) against the extensions built in-tree beforehand on the CPU.  Any step ending in a fault/abort/timeout stops the script.
set -u
R=$GRAFT_REPO_ROOT; T=${1:-run}; shift || true
STEPS=${*:-test bench precise prof}
cd $R
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2: stopping"; exit $1;; esac; }
for st in $STEPS; do
  case $st in
    test)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu_$T.log 2>&1
      rc=$?; echo pytest_rc=$rc; tail -4 gpurun_out/pytest_gpu_$T.log; fatal $rc pytest;;
    bench)
      timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
      rc=$?; echo bench_rc=$rc; cat gpurun_out/bench_$T.json; fatal $rc bench;;
    precise)
      timeout -k 10 240 python bench.py --precise --skip-fit > gpurun_out/bench_precise_$T.json 2>> gpurun_out/bench_$T.err
      rc=$?; echo benchp_rc=$rc; cat gpurun_out/bench_precise_$T.json; fatal $rc precise;;
    ablate)
      timeout -k 10 300 python tools/kmeans_ablate.py > gpurun_out/ablate_$T.json 2>&1
      rc=$?; echo ablate_rc=$rc; tail -2 gpurun_out/ablate_$T.json; fatal $rc ablate;;
    smoke)
      timeout -k 10 180 python __graft_entry__.py smoke > gpurun_out/smoke_$T.log 2>&1
      rc=$?; echo smoke_rc=$rc; tail -2 gpurun_out/smoke_$T.log; fatal $rc smoke;;
    pcabench)
      timeout -k 10 400 python benchmarks/bench_pca.py ${PCA_ARGS:-} > gpurun_out/bench_pca_$T.json 2> gpurun_out/bench_pca_$T.err
      rc=$?; echo pcabench_rc=$rc; cat gpurun_out/bench_pca_$T.json; tail -3 gpurun_out/bench_pca_$T.err; fatal $rc pcabench;;
    alsbench)
      timeout -k 10 600 python benchmarks/bench_als.py ${ALS_ARGS:-} > gpurun_out/bench_als_$T.json 2> gpurun_out/bench_als_$T.err
      rc=$?; echo alsbench_rc=$rc; cat gpurun_out/bench_als_$T.json; tail -3 gpurun_out/bench_als_$T.err; fatal $rc alsbench;;
    alsprof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/alsprof_$T -o run -- python3 $R/benchmarks/bench_als.py --ratings 20000000 --users 1000000 --items 100000 --iters 2 > $R/gpurun_out/alsprof_$T.log 2>&1)
      rc=$?; echo alsprof_rc=$rc; fatal $rc alsprof;;
    alsprof1b)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/alsprof1b_$T -o run -- python3 $R/benchmarks/bench_als.py --iters 2 > $R/gpurun_out/alsprof1b_$T.log 2>&1)
      rc=$?; echo alsprof1b_rc=$rc; fatal $rc alsprof1b;;
    pcaprof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pcaprof_$T -o run -- python3 $R/benchmarks/bench_pca.py --reps 2 > $R/gpurun_out/pcaprof_$T.log 2>&1)
      rc=$?; echo pcaprof_rc=$rc; fatal $rc pcaprof;;
    trace)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/trace_$T -o run -- python3 $R/bench.py --steps 20 --warmup 0 --skip-fit --skip-unpruned --no-separable-extra > $R/gpurun_out/trace_$T.log 2>&1)
      rc=$?; echo trace_rc=$rc; fatal $rc trace;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$T -o run -- python3 $R/bench.py --rows 20000000 --steps 5 --warmup 1 --skip-fit > $R/gpurun_out/prof_$T.log 2>&1)
      rc=$?; echo prof_rc=$rc; fatal $rc prof;;
    *)
      # any other step is a python script path relative to the repo, with output to a log
      timeout -k 10 600 python $st > gpurun_out/$(basename $st .py)_$T.log 2>&1
      rc=$?; echo "$st rc=$rc"; tail -5 gpurun_out/$(basename $st .py)_$T.log; fatal $rc $st;;
  esac
done
