#!/bin/bash
# usage: tools/gpu_steps.sh <tag> <step>...  (on the GPU box; extensions built in-tree beforehand)
# steps: test | bench | pca | als | alsrccl | alsprof | smoke | py:<script> ; any fault/timeout stops
set -u
R=$GRAFT_REPO_ROOT; T=$1; shift
cd $R; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
for st in "$@"; do
  case $st in
    test)
      timeout -k 10 800 python -u -m pytest ${PYTEST_TARGET:-tests} -m gpu -x -v ${PYTEST_EXTRA:-} --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1
      rc=$?; echo pytest_rc=$rc; grep -E "FAILED|passed|failed" gpurun_out/pytest_gpu_$T.log | tail -5; fatal $rc pytest;;
    bench)
      timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
      rc=$?; echo bench_rc=$rc; cat gpurun_out/bench_$T.json; fatal $rc bench;;
    pca)
      timeout -k 10 400 python benchmarks/bench_pca.py ${PCA_ARGS:-} > gpurun_out/bench_pca_$T.json 2> gpurun_out/bench_pca_$T.err
      rc=$?; echo pca_rc=$rc; cat gpurun_out/bench_pca_$T.json; tail -2 gpurun_out/bench_pca_$T.err; fatal $rc pca;;
    als)
      timeout -k 10 500 python benchmarks/bench_als.py --iters 3 ${ALS_ARGS:-} > gpurun_out/bench_als_$T.json 2> gpurun_out/bench_als_$T.err
      rc=$?; echo als_rc=$rc; cat gpurun_out/bench_als_$T.json; tail -2 gpurun_out/bench_als_$T.err; fatal $rc als;;
    alsrccl)
      timeout -k 10 500 python benchmarks/bench_als.py --force-rccl --iters 3 ${ALS_ARGS:-} > gpurun_out/bench_als_rccl_$T.json 2> gpurun_out/bench_als_rccl_$T.err
      rc=$?; echo alsrccl_rc=$rc; cat gpurun_out/bench_als_rccl_$T.json; tail -2 gpurun_out/bench_als_rccl_$T.err; fatal $rc alsrccl;;
    alsprof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/alsprof_$T -o run -- python3 $R/benchmarks/bench_als.py --iters 2 ${ALS_ARGS:-} > $R/gpurun_out/alsprof_$T.log 2>&1)
      rc=$?; echo alsprof_rc=$rc; fatal $rc alsprof;;
    pcaprof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pcaprof_$T -o run -- python3 $R/benchmarks/bench_pca.py --reps 1 ${PCA_ARGS:-} > $R/gpurun_out/pcaprof_$T.log 2>&1)
      rc=$?; echo pcaprof_rc=$rc; fatal $rc pcaprof;;
    kprof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kprof_$T -o run -- python3 $R/bench.py --steps 20 --warmup 1 --skip-fit --skip-unpruned --no-separable-extra --no-estimator ${BENCH_ARGS:-} > $R/gpurun_out/kprof_$T.log 2>&1)
      rc=$?; echo kprof_rc=$rc; fatal $rc kprof;;
    smoke)
      timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke_$T.log 2>&1
      rc=$?; echo smoke_rc=$rc; tail -2 gpurun_out/smoke_$T.log; fatal $rc smoke;;
    py:*)
      sc=${st#py:}
      timeout -k 10 600 python $sc > gpurun_out/$(basename $sc .py)_$T.log 2>&1
      rc=$?; echo "$sc rc=$rc"; tail -5 gpurun_out/$(basename $sc .py)_$T.log; fatal $rc $sc;;
  esac
done
