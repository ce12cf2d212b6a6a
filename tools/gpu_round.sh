#!/bin/bash
# usage: scratch/gpu_round.sh <tag>  -- build, gpu tests, bench (fast+precise), rocprof stats
set -u
R=$GRAFT_REPO_ROOT; T=${1:-run}
cd $R
python -m oap_mllib_amd.build > gpurun_out/build_$T.log 2>&1 || { echo build_failed; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu_$T.log 2>&1; echo pytest_rc=$?; tail -4 gpurun_out/pytest_gpu_$T.log
timeout -k 10 240 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err; echo bench_rc=$?; cat gpurun_out/bench_$T.json
timeout -k 10 240 python bench.py --precise --skip-fit > gpurun_out/bench_precise_$T.json 2>> gpurun_out/bench_$T.err; echo benchp_rc=$?; cat gpurun_out/bench_precise_$T.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$T -o run -- python3 $R/bench.py --rows 20000000 --steps 5 --warmup 1 --skip-fit > $R/gpurun_out/prof_$T.log 2>&1; echo prof_rc=$?
