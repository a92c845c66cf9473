set -e
mkdir -p gpurun_out/af
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 -L > gpurun_out/af/list.txt 2>&1 || true
for f in 8 20; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES -d gpurun_out/af/p1_f$f -o run -- python3 tools/x6_one.py 12800 3072 768 10 $f > gpurun_out/af/p1_f$f.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_WAVES -d gpurun_out/af/p2_f$f -o run -- python3 tools/x6_one.py 12800 3072 768 10 $f > gpurun_out/af/p2_f$f.log 2>&1
done
