set -o pipefail
mkdir -p gpurun_out
PROBE_SKINNY=1 timeout -k 10 300 python tools/probe/glds_probe.py 3,4,5,9,26,34 > gpurun_out/skinny.log 2>&1; rc=$?; cat gpurun_out/skinny.log; exit $rc
