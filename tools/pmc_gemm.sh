#!/bin/bash
# PMC passes for the top GEMMs of one training step (tools/gemm_census.py --replay):
# MFMA busy / wave-state counters (SQ + GRBM) and FETCH_SIZE / WRITE_SIZE, each in a
# run of its own (rocprofv3 does not split counters over passes). NTOP shapes.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_gemm
timeout -k 5 60 rocprofv3 -L > gpurun_out/pmc_gemm/counters_list.txt 2>&1 || true
SQ="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
# the five GEMMs with the largest total time per step (tools/gemm_census.py, round 2):
# M,N,K,amode,bmode[,pro_a]
KEYS=(${KEYS:-32,288,1048576,1,2 1048576,32,288,2,0 65536,4352,128,0,1 128,4352,65536,1,1 65536,128,4352,0,0,2})
for i in "${!KEYS[@]}"; do
  for pass in sq fetch write; do
    case $pass in
      sq) C="$SQ" ;;
      fetch) C="FETCH_SIZE" ;;
      write) C="WRITE_SIZE" ;;
    esac
    rm -rf gpurun_out/pmc_gemm/g${i}_$pass
    timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_gemm/g${i}_$pass -o run -- python tools/gemm_census.py --top 8 --replay-key ${KEYS[$i]} --reps 20 > gpurun_out/pmc_gemm/g${i}_$pass.log 2>&1
    # keep only the replayed GEMM dispatches (the full trace of the model step is ~10 MB)
    python tools/pmc_gemm_report.py --shrink gpurun_out/pmc_gemm/g${i}_$pass/run_counter_collection.csv
    rm -f gpurun_out/pmc_gemm/g${i}_$pass/run_agent_info.csv
    grep -o "replayed.*" gpurun_out/pmc_gemm/g${i}_$pass.log
    grep -v "^[WE]20" gpurun_out/pmc_gemm/g${i}_$pass.log > gpurun_out/pmc_gemm/g${i}_$pass.log.tmp || true
    mv gpurun_out/pmc_gemm/g${i}_$pass.log.tmp gpurun_out/pmc_gemm/g${i}_$pass.log
  done
done
python tools/pmc_gemm_report.py gpurun_out/pmc_gemm | tee gpurun_out/pmc_gemm/report.txt
