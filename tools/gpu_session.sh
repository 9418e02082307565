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
    testsall) run pytest_gpu 1100 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 900 python bench.py ;;
    benchq) run bench 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ;;
    rehearse2) run bench_rehearse2 900 env PG_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2 --warmup 1 ;;
    rehearse2c3) run bench_rehearse2c3 600 env PG_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --config c3 --steps 3 --warmup 1 ;;
    cover) run pytest_cover 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parse.py tests/test_gpu_rccl.py -k "k3 or early_split or build_host or rccl or last_chunk" -v --timeout 120 --timeout-method thread ;;
    dbgc3) run dbg_c3 400 env PG_LIB_NAME=libpangenome_hip_dbg.so python -u tools/dbg_host_c3.py 0 2 ;;
    missing) run dbg_missing 400 env PG_LIB_NAME=libpangenome_hip_dbg.so python -u tools/dbg_missing.py gpurun_out/missing.npz ;;
    bracketrep) run bracket_rep 600 python -u tools/corruption_bracket.py repeat ;;
    bracketcat) run bracket_cat 900 python -u tools/corruption_bracket.py cat ;;
    bracket) run bracket_sort 500 python -u tools/corruption_bracket.py sort ;;
    abc4dbg) run ab_c4dbg 600 env PG_DEBUG_BUILD=1 python -u tools/ab_k3.py --genomes 1000 --steps 2 --tune base ;;
    benchc4) run bench_c4 900 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-cli ;;
    benchsmall) run bench_small 600 python bench.py --config small --steps 5 --warmup 1 --no-cpu-baseline ;;
    benchc2) run bench_c2 600 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline ;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-window --no-cli --no-exchange --no-concurrent --no-c5 ;;
    pmcsq) bash tools/pmc_kernels.sh "k_emit_work|k_cover_p|k_build_range|k_emit\(|k_span_sum|k_split" sq ;;
    pmc) bash tools/pmc_kernels.sh "k_span_sum|k_emit|k_records|k_pack_fix|k_cover|k_short_emit|k_split|k_build_range|rocprim" tr traffic ;;
    parse) run pytest_parse 600 python -u -m pytest tests/test_gpu_parse.py -x -v --timeout 120 --timeout-method thread ;;
    parity) run pytest_parity 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -v --timeout 120 --timeout-method thread ;;
    abcover) run ab_cover 600 python -u tools/ab_k3.py --steps 12 --tune base --tune K3_COVER=2 ;;
    abhost) run ab_host 600 python -u tools/ab_k3.py --host --alt --steps 12 --tune base --tune H2D_CHUNK=134217728,H2D_TAIL=67108864 --tune H2D_CHUNK=201326592,H2D_TAIL=67108864 --tune H2D_CHUNK=134217728,H2D_TAIL=50331648 ;;
    abchunks) run ab_chunks 900 python -u tools/ab_k3.py --steps 10 --tune base --tune K3_HEAD=8 --tune K3_HEAD=8,K3_TAIL=6 --tune K3_CHUNKS=4,K3_HEAD=6,K3_TAIL=6 --tune K3_CHUNKS=4 --tune K3_CHUNKS=5,K3_HEAD=6,K3_TAIL=6 --tune K3_CHUNKS=2 ;;
    npz) run pytest_npz 600 python -u -m pytest tests/test_gpu_npz.py -x -v --timeout 300 --timeout-method thread ;;
    savebd) run save_bd 300 python -u tools/save_breakdown.py ;;
    findfr) run findfr 300 python -u tools/findfr_breakdown.py ;;
    tracewin) run trace_win 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/tw -o run --output-format csv -- python tools/ab_k3.py --host --steps 3 --tune base ;;
    abfin) run ab_fin 600 python -u tools/ab_k3.py --host --alt --steps 16 --tune base --tune base --env PG_EXP_FINISH_EARLY= --env PG_EXP_FINISH_EARLY=1 ;;
    c5diag) run c5_diag 900 env C5_DIAG=1 python -u tools/c5_forms.py 0:30 0:30 0:30 ;;
    c4cli) run c4_cli 900 env PG_TIMING_LOG=gpurun_out/c4_timing.jsonl python -u -m pytest tests/test_gpu_scale.py -k c4 -x -v --timeout 800 --timeout-method thread ;;
    c4ckpt) run c4_ckpt 900 python -u tools/c4_ckpt_times.py ;;
    c5rep) run c5_rep 900 python -u tools/c5_forms.py 0:30 0:30 0:30 0:30 2:30 ;;
    c5forms) run c5_forms 900 python -u tools/c5_forms.py ;;
    abdev) run ab_dev 600 python -u tools/ab_k3.py --steps 16 --tune base ;;
    ab) run ab_k3 600 python -u tools/ab_k3.py --steps 12 --tune base --tune K3_COVER=1 ;;
    listctr) run listctr 300 rocprofv3 -L ;;
    c5tests) run pytest_c5 1000 python -u -m pytest tests/test_gpu_c5.py -x -v -s --timeout 800 --timeout-method thread ;;
    c5probe) run c5_probe 600 python -u tools/c5_probe.py stream routed reps=4 ;;
    c5probeprof) run c5_probe_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5r -o run --output-format csv -- python -u tools/c5_probe.py stream routed reps=2 ;;
    newtests) run pytest_new 600 python -u -m pytest tests/test_gpu_parity.py -k "empty or device_resident" -x -v --timeout 120 --timeout-method thread ;;
    k1) run pytest_k1 600 python -u -m pytest tests/test_gpu_parse.py -k "-8] or -24] or -40] or one_read" -x -v --timeout 300 --timeout-method thread && run ab_k1 600 python -u tools/ab_k3.py --alt --steps 16 --tune base --tune K1=8 --tune K1=24 --tune K1=40 --tune K1=72 ;;
    k1prof) run k1_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k1 -o run --output-format csv -- python -u tools/ab_k3.py --alt --steps 6 --tune base --tune K1=8 --tune K1=24 ;;
    benchfull) run bench_full 900 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    c5pmc) for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_IDX_ACTIVE"; do i=$((${i:-0}+1)); run c5pmc_$i 300 timeout -s KILL 280 rocprofv3 --pmc $c --kernel-include-regex "k_cover_p|k_emit_work|k_route_scatter|k_route_emit|k_split|k_build_range|k_span_sum|k_emit" -d gpurun_out/c5pmc_$i -o pmc --output-format csv -- python -u tools/c5_probe.py stream routed reps=2; done ;;
    benchc5q) run bench_c5q 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cli --no-concurrent ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
