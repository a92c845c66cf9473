#!/bin/bash
# Interleaved same-box A/B of an environment switch on the default bench (cfg2 training iteration):
# ab_env.sh <VAR> <value A> <value B> [rounds] -> one "VAR=v value ms" line per run.
set -o pipefail
VAR=$1; A=$2; B=$3; R=${4:-2}
for i in $(seq 1 "$R"); do
  for v in "$A" "$B"; do
    env "$VAR=$v" timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-fwd --no-kbench \
      --no-cfg5 --no-cfg4 --no-host-input --no-hoist > gpurun_out/ab_run.log 2>&1 || { tail -5 gpurun_out/ab_run.log; exit 1; }
    python - "$VAR=$v" <<'PY'
import json, sys
line = [l for l in open("gpurun_out/ab_run.log") if l.startswith("{")][-1]
d = json.loads(line)
k = d.get("kernels", {})
print(sys.argv[1], round(d["value"], 1), d["ms_per_step"], {n: k[n]["device_ms"] for n in ("bilstm_bptt", "gemm_x6", "gemm") if n in k}, flush=True)
PY
  done
done
