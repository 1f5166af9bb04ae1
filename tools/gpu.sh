#!/bin/bash
# One parametrised driver for every GPU-box job (run through gpurun from the repo root).  Each
# GPU step runs under its own time limit and the first failure ends the script.
#
#   tools/gpu.sh smoke                          __graft_entry__.smoke()
#   tools/gpu.sh test [pytest args...]          GPU test suite (default: tests -m gpu)
#   tools/gpu.sh bench [N] [bench args...]      N x bench.py --steps 300 (default N=3), one line each
#   tools/gpu.sh ab KEY=V[,KEY=V] ...           bench.py under override sets (same box A/B)
#   tools/gpu.sh prof TAG [bench args...]       rocprofv3 kernel trace + step breakdown
#   tools/gpu.sh pmc TAG [filters...]           PMC passes over the bench step (kernel trace only)
#   tools/gpu.sh bytes TAG [bench args...]      FETCH_SIZE / WRITE_SIZE passes (roofline bytes)
#   tools/gpu.sh learn [learn_check args...]    tools/learn_check.py
#   tools/gpu.sh native [bench_native args...]  actor + learner loop (serial / concurrent)
#   tools/gpu.sh cfg2 [N] [steps]               main.py --cpu-actors N with an injected actor crash
#   tools/gpu.sh dp [N] [bench args...]         N-rank DP bench rehearsal sharing the one GPU
#
# Output goes under gpurun_out/ (merged back by gpurun); summaries worth keeping are copied into
# profiles/ by hand.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cmd=${1:-test}; shift || true

fail() { echo "FAIL: $1"; [ -f "$2" ] && tail -30 "$2"; exit 1; }

case "$cmd" in
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
      || fail smoke gpurun_out/smoke.log
    echo "smoke ok" ;;
  test)
    args=("$@"); [ ${#args[@]} -eq 0 ] && args=(tests -m gpu)
    timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread "${args[@]}" \
      > gpurun_out/pytest_gpu.txt 2>&1 || fail pytest gpurun_out/pytest_gpu.txt
    tail -2 gpurun_out/pytest_gpu.txt ;;
  bench)
    n=${1:-3}; shift || true
    for i in $(seq 1 "$n"); do
      timeout -k 10 180 python bench.py --steps 300 --warmup 30 "$@" > gpurun_out/bench_$i.log 2>&1 \
        || fail "bench $i" gpurun_out/bench_$i.log
      grep -h '^{' gpurun_out/bench_$i.log | python -c \
        "import sys,json; d=json.loads(sys.stdin.read()); print(d['config'].get('preset'), d['value'], d['ms_per_step'])"
    done ;;
  ab)
    for v in "$@"; do
      sets=(); IFS=, read -ra kvs <<< "$v"; for kv in "${kvs[@]}"; do [ -n "$kv" ] && sets+=(--set "$kv"); done
      timeout -k 10 180 python bench.py --steps 300 --warmup 30 "${sets[@]}" > gpurun_out/ab.log 2>&1 \
        || fail "ab [$v]" gpurun_out/ab.log
      echo "[$v] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log)"
    done ;;
  prof)
    tag=$1; shift
    rm -rf gpurun_out/prof_$tag
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -- \
      python bench.py --steps 20 --warmup 10 "$@" > gpurun_out/prof_$tag.log 2>&1 || fail "prof $tag" gpurun_out/prof_$tag.log
    grep -h '^{' gpurun_out/prof_$tag.log | cut -c1-120
    python tools/step_breakdown.py "gpurun_out/prof_$tag/*/*kernel_trace.csv" gpurun_out/$tag.txt 5 > /dev/null
    head -30 gpurun_out/$tag.txt ;;
  pmc)
    tag=$1; shift
    filters=("$@"); [ ${#filters[@]} -eq 0 ] && filters=(torso lstm gemm td_duel rmsprop)
    mkdir -p gpurun_out/pmc_$tag
    i=0
    for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS" \
               "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS" \
               "SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
               "SQ_INSTS_VMEM_RD SQ_INSTS_LDS_STORE SQ_INSTS_LDS_LOAD SQ_WAIT_INST_ANY" \
               "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
      i=$((i+1))
      timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc_$tag/p$i -- \
        python bench.py --steps 3 --warmup 2 > gpurun_out/pmc_$tag/p$i.log 2>&1 || fail "pmc pass $i" gpurun_out/pmc_$tag/p$i.log
    done
    python tools/pmc_summary.py "gpurun_out/pmc_$tag/p*/**/*counter_collection.csv" "${filters[@]}" \
      > gpurun_out/pmc_$tag/summary.txt
    head -60 gpurun_out/pmc_$tag/summary.txt ;;
  pmcmicro)
    # the pmc passes over a micro-benchmark instead of the bench step: pmcmicro TAG script args...
    tag=$1; shift
    mkdir -p gpurun_out/pmc_$tag
    i=0
    for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
               "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS" \
               "SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU" \
               "SQ_INSTS_VMEM_RD SQ_INSTS_LDS_STORE SQ_INSTS_LDS_LOAD SQ_WAIT_INST_ANY"; do
      i=$((i+1))
      timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc_$tag/p$i -- \
        python "$@" > gpurun_out/pmc_$tag/p$i.log 2>&1 || fail "pmcmicro pass $i" gpurun_out/pmc_$tag/p$i.log
    done
    python tools/pmc_summary.py "gpurun_out/pmc_$tag/p*/**/*counter_collection.csv" \
      > gpurun_out/pmc_$tag/summary.txt
    cat gpurun_out/pmc_$tag/summary.txt ;;
  bytes)
    # HBM-side byte counters per kernel (roofline input): FETCH_SIZE (3 TCC slots) and WRITE_SIZE
    # (2) in passes of their own, MFMA busy cycles beside them
    tag=$1; shift
    mkdir -p gpurun_out/bytes_$tag
    i=0
    for grp in "FETCH_SIZE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES" \
               "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
      i=$((i+1))
      timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/bytes_$tag/p$i -- \
        python bench.py --steps 3 --warmup 2 "$@" > gpurun_out/bytes_$tag/p$i.log 2>&1 || fail "bytes pass $i" gpurun_out/bytes_$tag/p$i.log
    done
    python tools/pmc_summary.py "gpurun_out/bytes_$tag/p*/**/*counter_collection.csv" \
      > gpurun_out/bytes_$tag/summary.txt
    head -40 gpurun_out/bytes_$tag/summary.txt ;;
  learn)
    timeout -k 10 300 python -u tools/learn_check.py "$@" > gpurun_out/learn.log 2>&1 || fail learn gpurun_out/learn.log
    grep -h '^{' gpurun_out/learn.log ;;
  cfg2)
    # BASELINE config 2: one GPU learner fed by N CPU actor processes (default 16), one injected
    # actor crash (restarted by the supervisor), metrics JSONL
    n=${1:-16}; steps=${2:-3000}
    R2D2_FAULTS="actor:3:crash_at=300,once=1" timeout -k 10 900 python -u main.py --mode native \
      --config pong --cpu-actors "$n" --steps "$steps" --metrics gpurun_out/cfg2_metrics.jsonl \
      > gpurun_out/cfg2.log 2>&1 || fail cfg2 gpurun_out/cfg2.log
    tail -n 3 gpurun_out/cfg2.log ;;
  dp)
    # multi-rank rehearsal on one GPU (gloo, ranks share the card): N ranks (default 4)
    n=${1:-4}; shift || true
    R2D2_BENCH_SHARED=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node "$n" --master-addr 127.0.0.1 --master-port 29531 bench.py --steps 20 \
      --warmup 5 --capacity 200000 "$@" > gpurun_out/dp.log 2>&1 || fail dp gpurun_out/dp.log
    grep -h '^{' gpurun_out/dp.log ;;
  native)
    timeout -k 10 240 python -u tools/bench_native.py "$@" >> gpurun_out/native.log 2>&1 \
      || fail native gpurun_out/native.log
    grep -h '^{' gpurun_out/native.log | tail -n 2 ;;
  *)
    echo "unknown command $cmd"; exit 2 ;;
esac
