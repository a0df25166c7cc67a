#!/bin/bash
# halo-tile 3x3 kernels (csrc/conv3x3.hip): parity tests (incl. bitwise vs the implicit
# GEMM), gbench A/B against the implicit GEMM (ACCUNET_CONV3_HALO=0), the suite, then
# bench lines fp32 / bf16 with the knob on and off
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_bf16_gpu.py tests/test_kernels_gpu.py -x -q --timeout 240 --timeout-method thread -k "eager or upsample_bwd24" > gpurun_out/c3_tests.log 2>&1 || { tail -30 gpurun_out/c3_tests.log; exit 1; }
tail -n 2 gpurun_out/c3_tests.log
: > gpurun_out/c3_ab.txt
for rep in 1; do
  for v in 1 0; do
    echo "== ACCUNET_CONV3_HALO=$v" >> gpurun_out/c3_ab.txt
    ACCUNET_CONV3_HALO=$v GB_ONLY=rspth timeout -k 10 120 tools/gbench 20 >> gpurun_out/c3_ab.txt 2>&1
  done
done
cat gpurun_out/c3_ab.txt
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 240 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -n 1 gpurun_out/gputests.log
for dt in fp32 bf16; do
  for v in 1 0; do
    ACCUNET_CONV3_HALO=$v timeout -k 10 400 python bench.py --dtype $dt --no-cpu-baseline > gpurun_out/bench_c3_${dt}_$v.log 2>&1
    echo "$dt halo=$v"; grep '^{"metric' gpurun_out/bench_c3_${dt}_$v.log | cut -c1-200
  done
done
grep -o '"before_steps": {[^}]*}' gpurun_out/bench_c3_fp32_1.log || true
