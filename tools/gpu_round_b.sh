#!/bin/bash
# Second half of the round profile pass (tools/gpu_round.sh split under one call's
# limit): FETCH_SIZE / WRITE_SIZE passes (separate runs) for K1's / K3's HBM traffic,
# tools/kbench and the single-stream step trace (the K1 instruction-level lab pass,
# tools/pmc_k1.sh, is not repeated)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --eager --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --eager --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1
python tools/save_profiles.py --shrink-pmc gpurun_out/pmc_fetch gpurun_out/pmc_write
echo "pmc done"
timeout -k 10 120 tools/kbench 20 > gpurun_out/kbench.txt 2>&1
echo "kbench done"
KGRID="splitk dw3x3" VARIANTS="ss:-" timeout -k 10 400 bash tools/prof_ab.sh > gpurun_out/prof_ss.log 2>&1
echo "single-stream trace done"
