# usage (GPU box): bash tools/gpu_r4prof.sh <tag>: kernel statistics + trace of the headline fit
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r4prof}
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_head_$T -o run -- python3 $GRAFT_REPO_ROOT/bench.py --warmup 1 --skip-fit --skip-unpruned --no-separable-extra --no-estimator --cpu-rows 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_head_$T.log 2>&1)
rc=$?; echo prof_rc=$rc
echo done
