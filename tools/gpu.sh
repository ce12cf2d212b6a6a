#!/bin/bash
# The one GPU-box runner (run through gpurun; extensions are built in-tree on the CPU first):
#
#   bash tools/gpu.sh <tag> <step>...
#
# Steps (each under its own time limit; a fault / abort / timeout stops the script there):
#   test       pytest -m gpu (PYTEST_TARGET, PYTEST_EXTRA)
#   smoke      __graft_entry__.smoke()
#   bench      python bench.py $BENCH_ARGS                     -> gpurun_out/bench_<tag>.json
#   cfg5       python bench.py --config kmeans_bf16 $CFG5_ARGS -> gpurun_out/cfg5_<tag>.json
#   pca | als | rec   benchmarks/bench_{pca,als,recommend}.py with $PCA_ARGS / $ALS_ARGS / $REC_ARGS
#   shard      the 8-GPU shard-size proxy on ONE GPU (100M/N rows, N = 1 2 4 8, 1-rank RCCL)
#   kprof | cfg5prof | pcaprof | alsprof   rocprofv3 --kernel-trace --stats of a bench
#   pmc:<probe.py>:<pass>   one PMC pass (counter set a|b|c|mem) over tools/<probe.py> $PROBE_ARGS
#   py:<script>             any python script, output to gpurun_out/<name>_<tag>.log
set -u
R=$GRAFT_REPO_ROOT; T=$1; shift
cd $R; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2: stopping"; exit $1;; esac; }
prof() {  # $1 = out name, $2 = time limit, rest = python args
  local O=$1 L=$2; shift 2
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 $L rocprofv3 --kernel-trace --stats \
     --output-format csv -d $R/gpurun_out/$O -o run -- python3 "$@" > $R/gpurun_out/$O.log 2>&1)
}
pmc_set() {
  case $1 in
    a) echo SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE;;
    b) echo SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE;;
    c) echo SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAVE_CYCLES GRBM_GUI_ACTIVE;;
    mem) echo TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE;;
    fetch) echo FETCH_SIZE GRBM_GUI_ACTIVE;;
  esac
}
for st in "$@"; do
  case $st in
    test)
      timeout -k 10 1100 python -u -m pytest ${PYTEST_TARGET:-tests} -m gpu -x -v ${PYTEST_EXTRA:-} --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1
      rc=$?; echo pytest_rc=$rc; grep -E "FAILED|passed|failed" gpurun_out/pytest_gpu_$T.log | tail -5; fatal $rc pytest;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$T.txt 2>&1
      rc=$?; echo smoke_rc=$rc; tail -1 gpurun_out/smoke_$T.txt; fatal $rc smoke;;
    bench)
      timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
      rc=$?; echo bench_rc=$rc; cat gpurun_out/bench_$T.json; fatal $rc bench;;
    cfg5)
      timeout -k 10 600 python bench.py --config kmeans_bf16 ${CFG5_ARGS:-} > gpurun_out/cfg5_$T.json 2> gpurun_out/cfg5_$T.err
      rc=$?; echo cfg5_rc=$rc; cat gpurun_out/cfg5_$T.json; tail -2 gpurun_out/cfg5_$T.err; fatal $rc cfg5;;
    pca|als|rec)
      b=$st; [ $st = rec ] && b=recommend
      eval "A=\${$(echo $st | tr a-z A-Z)_ARGS:-}"
      timeout -k 10 600 python benchmarks/bench_$b.py $A > gpurun_out/bench_${st}_$T.json 2> gpurun_out/bench_${st}_$T.err
      rc=$?; echo ${st}_rc=$rc; cat gpurun_out/bench_${st}_$T.json; tail -2 gpurun_out/bench_${st}_$T.err; fatal $rc $st;;
    shard)
      for n in 1 2 4 8; do
        timeout -k 10 300 python bench.py --rows $((100000000 / n)) --force-rccl --cpu-rows 0 --no-estimator --no-separable-extra ${BENCH_ARGS:-} > gpurun_out/shard_${T}_n$n.json 2> gpurun_out/shard_${T}_n$n.err
        rc=$?; echo shard_n${n}_rc=$rc; fatal $rc shard$n
      done;;
    kprof)
      prof kprof_$T 300 $R/bench.py --warmup 1 --skip-fit --skip-unpruned --no-separable-extra --no-estimator --cpu-rows 0 ${BENCH_ARGS:-}
      rc=$?; echo kprof_rc=$rc; fatal $rc kprof;;
    cfg5prof)
      prof cfg5prof_$T 600 $R/bench.py --config kmeans_bf16 --warmup 0 --steps 4 --skip-fit --skip-unpruned --no-separable-extra --no-estimator --cpu-rows 0 ${CFG5_ARGS:-}
      rc=$?; echo cfg5prof_rc=$rc; fatal $rc cfg5prof;;
    pcaprof)
      prof pcaprof_$T 300 $R/benchmarks/bench_pca.py --reps 1 ${PCA_ARGS:-}
      rc=$?; echo pcaprof_rc=$rc; fatal $rc pcaprof;;
    alsprof)
      prof alsprof_$T 400 $R/benchmarks/bench_als.py --iters 2 ${ALS_ARGS:-}
      rc=$?; echo alsprof_rc=$rc; fatal $rc alsprof;;
    pmc:*)
      IFS=: read -r _ probe pass <<< "$st"
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${T}_${pass} -o run --pmc $(pmc_set $pass) -- python3 $R/tools/$probe ${PROBE_ARGS:-} > $R/gpurun_out/pmc_${T}_${pass}.log 2>&1)
      rc=$?; echo pmc_${pass}_rc=$rc; fatal $rc pmc_$pass;;
    py:*)
      sc=${st#py:}
      timeout -k 10 600 python $sc ${PY_ARGS:-} > gpurun_out/$(basename $sc .py)_$T.log 2>&1
      rc=$?; echo "$sc rc=$rc"; tail -5 gpurun_out/$(basename $sc .py)_$T.log; fatal $rc $sc;;
    *) echo "unknown step $st"; exit 2;;
  esac
done
echo done
