cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u tools/kmeans_img_probe.py 100000000 8 5 old,-1,0,2,3,5,9,17,33,65,129,29,221 > gpurun_out/img_probe_r4a.jsonl 2> gpurun_out/img_probe_r4a.err && \
timeout -k 10 600 python -u -m pytest tests/test_kmeans_gpu.py -x -v --timeout 120 --timeout-method thread -k "image or pruning or lean_pass or batched" > gpurun_out/pytest_img_r4a.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_r4a.json 2> gpurun_out/bench_r4a.err
echo rc=$?
