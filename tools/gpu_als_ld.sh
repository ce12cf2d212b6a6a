# usage (GPU box): bash tools/gpu_als_ld.sh <tag>: ALS 1B with the factor pitch 112 vs 128
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-alsld}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2: stopping"; exit $1;; esac; }
for ld in 128 112; do
OAP_ALS_LD=$ld timeout -k 10 400 python benchmarks/bench_als.py --cpu-ratings 0 > gpurun_out/${T}_ld$ld.json 2> gpurun_out/${T}_ld$ld.err
rc=$?; echo ld${ld}_rc=$rc; fatal $rc ld$ld
done
