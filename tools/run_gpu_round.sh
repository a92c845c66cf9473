#!/bin/bash
# One GPU session: parity tests, smoke, DP rehearsal (2 ranks on one GPU over gloo), bench, rocprof stats.
# Any step that faults, aborts or times out ends the session (nothing else touches the GPU after it).
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r02}

step() {   # step <name> <timeout> <log> cmd...
  local name=$1 t=$2 log=$3; shift 3
  timeout -k 10 "$t" "$@" > "$log" 2>&1
  local rc=$?
  echo "${name}_rc=$rc"
  case $rc in
    124|134|137|139) echo "stopping after $name (rc=$rc)"; tail -20 "$log"; exit $rc ;;
  esac
  return 0
}

[ "${TESTS:-1}" = "1" ] && step tests 400 gpurun_out/tests_$TAG.log python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread
grep -E "passed|failed" gpurun_out/tests_$TAG.log | tail -3
[ "${TESTS:-1}" = "1" ] && step smoke 200 gpurun_out/smoke_$TAG.log python -c "import __graft_entry__ as g; g.smoke()"
if [ "${DP:-0}" = "1" ]; then
  DASA_LSTM_MODE=1 step dp 400 gpurun_out/dp2_$TAG.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 0 --backend gloo \
    --same-device --no-fwd --no-profile --max-action 4
fi
[ "${BENCH:-1}" = "1" ] && step bench 600 gpurun_out/bench_$TAG.log python bench.py --steps ${STEPS:-3} --warmup 1
tail -1 gpurun_out/bench_$TAG.log
if [ "${PROF:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  step prof 600 gpurun_out/profrun_$TAG.log rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-fwd \
    --no-cfg5 --no-kbench
  # keep only the summaries (the full kernel trace is far larger than gpurun's copy-back limit)
  find gpurun_out/prof_$TAG \( -name "*kernel_trace*" -o -name "*.db" \) -delete 2>/dev/null
  find gpurun_out/prof_$TAG -type f
  python tools/prof_compare.py gpurun_out/prof_$TAG/run_kernel_stats.csv gpurun_out/profrun_$TAG.log \
    > gpurun_out/prof_compare_$TAG.txt
  head -20 gpurun_out/prof_compare_$TAG.txt
fi
