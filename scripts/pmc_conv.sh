#!/bin/bash
# rocprofv3 PMC passes over the conv kernels of the hottest shapes (one pass per counter
# group: <= 8 SQ counters, FETCH_SIZE and WRITE_SIZE in separate passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=${OUT:-gpurun_out/pmc_conv}
mkdir -p $OUT
export TMPDIR=/tmp
SHAPES=${SHAPES:-stem seg l1 proj960}
KIND=${KIND:-all}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
for s in $SHAPES; do
  for pass in 1 2; do
    eval "CTRS=\$P$pass"
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT/${s}_p$pass -o run --output-format csv \
      -- python scripts/conv_pmc.py $s $KIND 5 > $OUT/${s}_p$pass.log 2>&1 || { echo "pass $s/$pass failed"; exit 1; }
  done
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/${s}_fetch -o run --output-format csv \
    -- python scripts/conv_pmc.py $s $KIND 5 > $OUT/${s}_fetch.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/${s}_write -o run --output-format csv \
    -- python scripts/conv_pmc.py $s $KIND 5 > $OUT/${s}_write.log 2>&1 || exit 1
done
echo done
