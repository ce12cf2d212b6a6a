cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_kmeans_gpu.py tests/test_als_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_r4d.log 2>&1 ; \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/trace_bench_r4d -o run -- python3 $GRAFT_REPO_ROOT/bench.py --warmup 0 --skip-fit --skip-unpruned --no-separable-extra --no-estimator > $GRAFT_REPO_ROOT/gpurun_out/trace_bench_r4d.log 2>&1) && \
bash tools/pmc_img.sh pmcimg_r4d old,-1 20000000
echo rc=$?
