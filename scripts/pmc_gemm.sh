#!/bin/bash
# rocprofv3 PMC passes over e2ep_gemm for one shape: SHAPE="M N K ak bk" [FORCE="tm tn s"]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=${OUT:-gpurun_out/pmc_gemm}
NAME=${NAME:-ffn1}
SHAPE=${SHAPE:-"2048 2048 258 1 1"}
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
for pass in 1 2; do
  eval "CTRS=\$P$pass"
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT/${NAME}_p$pass -o run --output-format csv \
    -- python scripts/gemm_pmc.py $SHAPE 5 $FORCE > $OUT/${NAME}_p$pass.log 2>&1 || { echo "pass $pass failed"; exit 1; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/${NAME}_fetch -o run --output-format csv \
  -- python scripts/gemm_pmc.py $SHAPE 5 $FORCE > $OUT/${NAME}_fetch.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/${NAME}_write -o run --output-format csv \
  -- python scripts/gemm_pmc.py $SHAPE 5 $FORCE > $OUT/${NAME}_write.log 2>&1 || exit 1
echo done
