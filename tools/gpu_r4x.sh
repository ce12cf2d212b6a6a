# usage (GPU box): bash tools/gpu_r4x.sh <tag>: kernel statistics of config 5 (k=1000, bf16, 1B rows)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r4x}
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_cfg5_$T -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config kmeans_bf16 --steps 4 --warmup 0 --skip-fit --skip-unpruned --no-separable-extra --no-estimator --cpu-rows 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_cfg5_$T.log 2>&1)
rc=$?; echo prof_rc=$rc
echo done
