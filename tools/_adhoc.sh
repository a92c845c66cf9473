set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 200 --timeout-method thread -k "finetune or lxrt" > gpurun_out/t_ft.log 2>&1; rc=$?; tail -30 gpurun_out/t_ft.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-kbench > gpurun_out/b_n.log 2>&1; rc=$?; tail -1 gpurun_out/b_n.log | python -c '
import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d.get("fwd_value")); print({k:(v["launches"], v["device_ms"], v["avg_launch_us"], v["frac"]) for k,v in d["kernels"].items()})'; exit $rc
