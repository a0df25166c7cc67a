#!/bin/bash
# development pass: the streaming-kernel / model / bf16 GPU suites, then the bench with
# both K1 tile heights (ACCUNET_DW_OS16 A/B); each GPU step under its own time limit,
# the first failure ends the pass
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 700 python -u -m pytest ${TESTS:-tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_bf16_gpu.py} -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_t.log 2>&1 || { tail -30 gpurun_out/gpu_t.log; exit 1; }
  tail -n 2 gpurun_out/gpu_t.log
fi
pick='"value": [0-9.]*|"kernel": "[a-z_+0-9]*", "shape": "[0-9x]*", "avg_us": [0-9.]*|"frac": [0-9.]*'
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_t.log 2>&1
grep -oE "$pick" gpurun_out/bench_t.log | head -12
if [ -n "${AB:-}" ]; then
  env $AB timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > gpurun_out/bench_tb.log 2>&1
  echo "--- $AB"; grep -oE "$pick" gpurun_out/bench_tb.log | head -12
fi
