#!/bin/bash
# bf16x6 tile-order A/B (DASA_X6_GROUP): isolated time per launch and FETCH_SIZE per launch per group
# setting on the language-stack shapes (tools/x6_one.py back to back).
set -o pipefail
OUT=gpurun_out/x6group
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for S in ${SHAPES:-12800,3072,768 12800,2304,768 12800,768,3072}; do
  IFS=, read M N K <<< "$S"
  for G in ${X6_GROUP_LIST:-4 8 16 1 -2 -4 -8}; do
    DASA_X6_GROUP=$G timeout -k 10 60 python tools/x6_one.py $M $N $K 20 > $OUT/t_${M}_${N}_${K}_g$G.txt 2>&1 || exit 1
    DASA_X6_GROUP=$G timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "f32x6" --output-format csv -d $OUT/p_${M}_${N}_${K}_g$G -o run -- python3 tools/x6_one.py $M $N $K 10 > $OUT/r_${M}_${N}_${K}_g$G.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "pmc $S g$G rc=$rc"; exit $rc; }
    F=$(find $OUT/p_${M}_${N}_${K}_g$G -name "*counter_collection.csv" | head -1)
    FS=$(python tools/pmc_kernels.py $F | grep -o "'FETCH_SIZE': [0-9]*" | grep -o "[0-9]*$")
    find $OUT/p_${M}_${N}_${K}_g$G -name "*.csv" -delete
    echo "$M x $N x $K group $G: $(grep -o '[0-9.]* us .*' $OUT/t_${M}_${N}_${K}_g$G.txt)  fetch_MB=$(python -c "print(round($FS*2048/1e6,1))")"
  done
done
