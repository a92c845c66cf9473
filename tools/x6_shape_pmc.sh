#!/bin/bash
# Per-shape HBM traffic of the bf16x6 GEMM on LONG dispatches: each shape of the
# training iteration's top gemm_x6 list runs back to back (tools/x6_one.py, >= 100 us per dispatch, so
# the counter window's fixed overhead is small), one rocprofv3 --pmc pass for FETCH_SIZE and one for
# WRITE_SIZE per shape. tools/x6_shape_summary.py turns them into bytes per launch (FETCH_SIZE x 2 KiB
# per the guide's gfx950 correction, WRITE_SIZE x 1 KiB) against the algorithmic 4MK + 6KN + 4MN.
set -o pipefail
OUT=gpurun_out/x6shape
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
SHAPES=${SHAPES:-"12800,3072,768 12800,2304,768 12800,768,3072 1600,3072,768 1600,768,3072 720,768,3072 1400,1024,4096"}
for S in $SHAPES; do
  IFS=, read M N K <<< "$S"
  timeout -k 10 60 python tools/x6_one.py $M $N $K 20 > $OUT/plain_${M}_${N}_${K}.txt 2>&1 || exit 1
  cat $OUT/plain_${M}_${N}_${K}.txt
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex "f32x6" --output-format csv -d $OUT/p_${M}_${N}_${K}_$C -o run -- python3 tools/x6_one.py $M $N $K 10 > $OUT/run_${M}_${N}_${K}_$C.log 2>&1
    rc=$?
    [ $rc -ne 0 ] && { echo "pmc $S $C rc=$rc"; tail -5 $OUT/run_${M}_${N}_${K}_$C.log; exit $rc; }
    F=$(find $OUT/p_${M}_${N}_${K}_$C -name "*counter_collection.csv" | head -1)
    python tools/pmc_kernels.py $F > $OUT/pmc_${M}_${N}_${K}_$C.txt
    find $OUT/p_${M}_${N}_${K}_$C -name "*.csv" -delete
  done
done
python tools/x6_shape_summary.py $OUT
