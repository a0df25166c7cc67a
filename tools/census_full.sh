set -e -o pipefail
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 300 python tools/gemm_census.py --top 200 > gpurun_out/census_full.txt 2>&1
