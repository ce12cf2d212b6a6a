# usage (GPU box): bash tools/gpu_r4h.sh <tag>; fused-scan configs A/B + recommend tests
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r4h}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_recommend_gpu.py tests/test_kmeans_gpu.py -v --timeout 120 --timeout-method thread -k "recommend or topk or slabs or fewer or pruning or image or bitwise" > gpurun_out/pytest_$T.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/pytest_$T.log; fatal $rc pytest
for c in 1 0; do
OAP_KMEANS_SCAN_CFG=$c timeout -k 10 300 python bench.py --cpu-rows 0 --no-estimator > gpurun_out/bench_${T}_scfg$c.json 2> gpurun_out/bench_${T}_scfg$c.err
rc=$?; echo bench_cfg${c}_rc=$rc; fatal $rc bench
done
(cd /tmp && export TMPDIR=/tmp && OAP_KMEANS_SCAN_CFG=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/trace_bench_$T -o run -- python3 $GRAFT_REPO_ROOT/bench.py --warmup 0 --skip-fit --skip-unpruned --no-separable-extra --no-estimator --cpu-rows 0 > $GRAFT_REPO_ROOT/gpurun_out/trace_bench_$T.log 2>&1)
rc=$?; echo trace_rc=$rc; fatal $rc trace
echo done
