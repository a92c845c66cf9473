set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_l.log 2>&1; rc=$?; tail -3 gpurun_out/t_l.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -m dasa_amd.kbench 20 256 > gpurun_out/kb_l.log 2>&1; rc=$?; cat gpurun_out/kb_l.log | python -c '
import json,sys
t=sys.stdin.read(); d=json.loads(t[t.index("{"):])
for k,v in d.items(): print(k, {b: (x["us"], x["GB/s"]) for b,x in v.items()})'; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_l.log 2>&1; rc=$?; tail -1 gpurun_out/b_l.log | python -c '
import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d.get("fwd_value")); print({k:(v["avg_launch_us"], v["achieved"], v["frac"]) for k,v in d["kernels"].items()})'; exit $rc
