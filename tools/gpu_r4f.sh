# usage (GPU box): bash tools/gpu_r4f.sh <tag>; stops on any fault/abort/timeout
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r4f}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2: stopping"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/pytest_$T.log; fatal $rc pytest
timeout -k 10 300 python -u tools/kmeans_img_probe.py 100000000 8 5 old,-1,0,2 > gpurun_out/img_probe_$T.jsonl 2> gpurun_out/img_probe_$T.err
rc=$?; echo probe_rc=$rc; fatal $rc probe
timeout -k 10 300 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; echo bench_rc=$rc; fatal $rc bench
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/trace_bench_$T -o run -- python3 $GRAFT_REPO_ROOT/bench.py --warmup 0 --skip-fit --skip-unpruned --no-separable-extra --no-estimator --cpu-rows 0 > $GRAFT_REPO_ROOT/gpurun_out/trace_bench_$T.log 2>&1)
rc=$?; echo trace_rc=$rc; fatal $rc trace
echo done
