# usage (GPU box): bash tools/gpu_r4als.sh <tag>: ALS 1B-rating bench + config 5 bench (final state)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r4als}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2: stopping"; exit $1;; esac; }
timeout -k 10 500 python benchmarks/bench_als.py --cpu-ratings 0 > gpurun_out/bench_als_$T.json 2> gpurun_out/bench_als_$T.err
rc=$?; echo als_rc=$rc; fatal $rc als
timeout -k 10 600 python bench.py --config kmeans_bf16 --cpu-rows 0 --no-estimator --skip-unpruned > gpurun_out/bench_cfg5_$T.json 2> gpurun_out/bench_cfg5_$T.err
rc=$?; echo cfg5_rc=$rc; fatal $rc cfg5
echo done
