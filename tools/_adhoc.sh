set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 200 --timeout-method thread -k "gemm_bf16" > gpurun_out/t_bf16.log 2>&1; rc=$?; tail -3 gpurun_out/t_bf16.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/probe/bf16_probe.py > gpurun_out/bf16.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/bf16.log; exit $rc
