#!/bin/bash
# K-Means lean pass: register-resident plane (variant 11) vs the LDS plane — tests, then the
# headline bench both ways (tools/gpu_steps.sh steps; any fault/timeout stops)
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${1:-r3l}
OAP_KMEANS_REG_PLANE=1 PYTEST_TARGET=tests/test_kmeans_gpu.py bash tools/gpu_steps.sh ${T}reg test || exit $?
BENCH_ARGS="--no-separable-extra --no-estimator --skip-unpruned" bash tools/gpu_steps.sh ${T}lds bench || exit $?
OAP_KMEANS_REG_PLANE=1 BENCH_ARGS="--no-separable-extra --no-estimator --skip-unpruned" bash tools/gpu_steps.sh ${T}reg bench || exit $?
