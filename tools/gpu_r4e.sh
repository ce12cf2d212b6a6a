cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_r4e.log 2>&1 && \
timeout -k 10 300 python -u tools/kmeans_img_probe.py 100000000 8 5 old,-1,0,2 > gpurun_out/img_probe_r4e.jsonl 2> gpurun_out/img_probe_r4e.err && \
timeout -k 10 300 python bench.py > gpurun_out/bench_r4e.json 2> gpurun_out/bench_r4e.err && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/trace_bench_r4e -o run -- python3 $GRAFT_REPO_ROOT/bench.py --warmup 0 --skip-fit --skip-unpruned --no-separable-extra --no-estimator > $GRAFT_REPO_ROOT/gpurun_out/trace_bench_r4e.log 2>&1)
echo rc=$?
