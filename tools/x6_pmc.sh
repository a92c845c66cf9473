set -o pipefail
OUT=gpurun_out/x6pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 60 python tools/x6_one.py 12800 3072 768 20 > $OUT/plain.txt 2>&1 || exit 1
n=0
for CTRS in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM_RD"; do
  n=$((n + 1))
  timeout -s KILL 90 rocprofv3 --pmc $CTRS --kernel-include-regex "f32x6" --output-format csv -d $OUT/p$n -o run -- python3 tools/x6_one.py 12800 3072 768 5 > $OUT/p${n}_run.log 2>&1
  rc=$?
  echo "pass$n rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $OUT/p${n}_run.log; exit $rc; }
  F=$(find $OUT/p$n -name "*counter_collection.csv" | head -1)
  python tools/pmc_kernels.py $F > $OUT/p$n.txt
  find $OUT/p$n -name "*.csv" -delete
done
cat $OUT/plain.txt $OUT/p1.txt $OUT/p2.txt
