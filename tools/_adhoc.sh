set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_n.log 2>&1; rc=$?; tail -3 gpurun_out/t_n.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-kbench > gpurun_out/b_n.log 2>&1; rc=$?; tail -1 gpurun_out/b_n.log | python -c '
import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d.get("fwd_value")); print({k:(v["launches"], v["device_ms"], v["avg_launch_us"], v["frac"]) for k,v in d["kernels"].items()})'; exit $rc
