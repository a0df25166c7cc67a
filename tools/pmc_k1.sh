#!/bin/bash
# Instruction-level PMC of K1 (the HANC depthwise forward, 16x256x256x96 fp32) beside
# arithmetic-free lab kernels of the same access shape and the K1 candidates of
# tools/k1lab2: SQ wave-state / instruction counters, TA back-pressure, GRBM clock, and
# FETCH_SIZE / WRITE_SIZE -- each counter set in a rocprofv3 --pmc run of its own (no
# splitting over passes). Needs tools/k1lab and tools/k1lab2 built (make -C tools).
#   bash tools/pmc_k1.sh; python tools/pmc_k1_report.py gpurun_out/pmc_k1
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_k1
rm -rf $OUT && mkdir -p $OUT
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE"
  "SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
# k1lab: only the arithmetic-free structures worth comparing (copy, tile_reg, tile_lds, strip)
RE_LAB="copy_x4|tile_reg|tile_lds|strip_lds"
for prog in k1lab2 k1lab; do
  RE=".*"; [ $prog = k1lab ] && RE="$RE_LAB"
  for i in "${!PASSES[@]}"; do
    timeout -s KILL 90 rocprofv3 --pmc ${PASSES[$i]} --kernel-include-regex "$RE" --output-format csv \
      -d $OUT/${prog}_p$i -o run -- tools/$prog 5 > $OUT/${prog}_p$i.log 2>&1
    rm -f $OUT/${prog}_p$i/run_agent_info.csv
  done
done
python tools/pmc_k1_report.py $OUT | tee $OUT/report.txt
