#!/bin/bash
# the whole -m gpu suite at the final sources
set -e -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -q -m gpu --timeout 560 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
tail -n 2 gpurun_out/gputests.log
