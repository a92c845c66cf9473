set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu > gpurun_out/k4.log 2>&1; echo k_rc=$?
timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/gemm2.log 2>&1; echo g_rc=$?
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench3.log 2>&1; echo bench_rc=$?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o r01 -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-fwd > gpurun_out/prof1.log 2>&1; echo prof_rc=$?
