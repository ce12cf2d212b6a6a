cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u tools/kmeans_img_probe.py 100000000 8 5 old,-1,0,197,201,213,229,196 > gpurun_out/img_probe_r4b.jsonl 2> gpurun_out/img_probe_r4b.err && \
timeout -k 10 600 python -u -m pytest tests/test_kmeans_gpu.py tests/test_als_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_r4b.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_r4b.json 2> gpurun_out/bench_r4b.err && \
bash tools/pmc_img.sh pmcimg_r4b old,-1 20000000
echo rc=$?
