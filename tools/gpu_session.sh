#!/bin/bash
# One GPU session: parity tests, smoke, bench. Each GPU step has its own time
# limit; a fault/abort/timeout ends the session (exit codes other than 0/1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    testsall) run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 900 python bench.py ;;
    benchq) run bench 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ;;
    benchsmall) run bench_small 600 python bench.py --config small --steps 5 --warmup 1 --no-cpu-baseline ;;
    benchc2) run bench_c2 600 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline ;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-window ;;
    pmc) for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" TCC_EA0_ATOMIC_sum "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"; do
           tag=$(echo $ctr | tr ' ' '_')
           run pmc_$tag 600 rocprofv3 --pmc $ctr --kernel-include-regex "k_insert|k_reduce|k_emit|k_span_sum" -d gpurun_out/pmc_$tag -o pmc --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
         done ;;
    listctr) run listctr 300 rocprofv3 -L ;;
    chunksweep) for n in 1 2 3 4; do
           PG_K3_CHUNKS=$n run bench_chunks_$n 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
         done ;;
    k5sweep) for cfg in "2 4096" "2 2304" "1 4096" "1 8192" "4 2048" "4 1024"; do
           set -- $cfg
           PG_K5_RU=$1 PG_K5_GRID=$2 run bench_k5_$1_$2 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
         done ;;
    ovsweep) for cfg in ${OVCFG:-"4 8192 512"}; do
           set -- $cfg
           PG_K3_CHUNKS=$1 PG_K3_COVPAD=$2 PG_K3_WGRID=$3 run bench_ov_$1_$2_$3 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
         done ;;
    loadsweep) for l in 0.25 0.5 0.7; do
           PG_BUCKET_LOAD=$l run bench_load_$l 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
         done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
