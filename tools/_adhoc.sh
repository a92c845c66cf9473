set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 200 --timeout-method thread -k "bf16" > gpurun_out/t_bf16.log 2>&1; rc=$?; tail -30 gpurun_out/t_bf16.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/probe/bf16_probe.py > gpurun_out/bf16.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/bf16.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --cfg5-only > gpurun_out/b_cfg5.log 2>&1; rc=$?; tail -1 gpurun_out/b_cfg5.log; exit $rc
