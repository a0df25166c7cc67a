set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -q -x --timeout 300 --timeout-method thread > gpurun_out/dist.log 2>&1 || { tail -40 gpurun_out/dist.log; exit 1; }
tail -3 gpurun_out/dist.log
timeout -k 10 400 python bench.py > gpurun_out/bench_parity.log 2>&1 || { tail -30 gpurun_out/bench_parity.log; exit 1; }
tail -1 gpurun_out/bench_parity.log
