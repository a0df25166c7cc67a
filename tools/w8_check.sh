#!/bin/bash
# the world-8 gloo rehearsal on the one GPU (tests/test_dist_gpu.py::test_world8_...)
set -e -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -x -v -s -m gpu -k "world8 or world4_buckets" --timeout 560 --timeout-method thread > gpurun_out/w8.log 2>&1 || { tail -60 gpurun_out/w8.log; exit 1; }
grep -E "fp64 mean|passed|PASSED" gpurun_out/w8.log | tail -20
