#!/bin/bash
# Measurement session for one round (run on the GPU box from the repo root):
#   1. bench.py's training iteration with its per-launch HIP-event kernel table (--shapes);
#   2. rocprofv3 --kernel-trace --stats of the TIMED path alone (graph replay on, no profile step) and the
#      per-family comparison of its average launch durations with the bench table (tools/prof_compare.py);
#   3. three rocprofv3 --pmc passes over one iteration (FETCH_SIZE / WRITE_SIZE / MFMA busy + clock),
#      summarised per family by tools/pmc_summary.py (HBM bytes with the gfx950 FETCH_SIZE x2
#      correction, MFMA-busy fraction).
# Every GPU step has its own time limit; a fault / abort / timeout ends the session.
set -o pipefail
TAG=${TAG:-r03}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
BENCH_ARGS="--no-cfg5 --no-cfg4 --no-aug --no-kbench --no-cpu-baseline --no-fwd --no-hoist --no-host-input"

step() {   # step <name> <timeout> <log> cmd...
  local name=$1 t=$2 log=$3; shift 3
  timeout -k 10 -s KILL "$t" "$@" > "$log" 2>&1
  local rc=$?
  echo "${name}_rc=$rc"
  case $rc in
    124|134|137|139) echo "stopping after $name (rc=$rc)"; tail -20 "$log"; exit $rc ;;
  esac
  return 0
}

if [ "${SKIP_STATS:-0}" != "1" ]; then   # SKIP_STATS=1: the PMC passes only (a second session)
step bench 400 $OUT/bench.log python bench.py --steps 3 --warmup 1 --shapes 40 $BENCH_ARGS
grep '^{"metric"' $OUT/bench.log | tail -1 > $OUT/bench.json
step stats 500 $OUT/stats_run.log rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-profile $BENCH_ARGS
# GPU busy / idle over the last timed iteration (union of kernel intervals; tools/timeline.py)
TRACE=$(find $OUT/stats -name "*kernel_trace.csv" | head -1)
[ -n "$TRACE" ] && python tools/timeline.py "$TRACE" ${ITER_MS:-420} > $OUT/timeline_last_iter.txt 2>&1
find $OUT/stats \( -name "*kernel_trace*" -o -name "*.db" \) -delete 2>/dev/null
STATS=$(find $OUT/stats -name "run_kernel_stats.csv" | head -1)
[ -n "$STATS" ] && python tools/prof_compare.py "$STATS" $OUT/bench.json > $OUT/prof_compare.txt && cat $OUT/prof_compare.txt
fi
REGEX='gemm|mha|bilstm|attn_|ln_fwd|policy_head|ew4|gather|adain'
# PMC per workload (each summary is attached only to its own workload's bench numbers, dasa_amd/prof.py
# PMC_FILES): cfg2 = the timed training iteration, cfg5 = configs[4]'s B=256 rollouts (bf16 + fp32),
# cfg4 = the README finetune iteration
for W in ${PMC_WORKLOADS:-cfg2 cfg5 cfg4}; do
  case $W in
    cfg2) WARGS="--steps 1 --warmup 1 --no-profile $BENCH_ARGS" ;;
    *) WARGS="--only $W" ;;
  esac
  n=0
  for CTRS in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES"; do
    n=$((n + 1))
    step pmc_${W}_$n 400 $OUT/pmc_${W}_${n}_run.log rocprofv3 --pmc $CTRS --kernel-include-regex "$REGEX" \
      --output-format csv -d $OUT/pmc_${W}_$n -o run -- python3 bench.py $WARGS
  done
  P1=$(find $OUT/pmc_${W}_1 -name "*counter_collection.csv" | head -1)
  P2=$(find $OUT/pmc_${W}_2 -name "*counter_collection.csv" | head -1)
  P3=$(find $OUT/pmc_${W}_3 -name "*counter_collection.csv" | head -1)
  python tools/pmc_summary.py $OUT/pmc_${W}.json $P1 $P2 $P3
  find $OUT -name "*counter_collection.csv" -delete 2>/dev/null
done
# the raw per-dispatch counter CSVs are large: keep the summaries only
find $OUT -name "*counter_collection.csv" -delete 2>/dev/null
find $OUT \( -name "*kernel_trace*" -o -name "*.db" \) -delete 2>/dev/null
ls -R $OUT | head -40
