#!/bin/bash
# round-4 final tree (wide-kernel loads spread over the MFMAs): every GPU test, smoke,
# the default bench line with its aux legs, rocprof stats, GEMM SQ counters.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4s; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_measure.sh r4s smoke bench prof && \
  bash tools/pmc_cmd.sh $O/pmc_gemm bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-aux --kernel-timing-steps 0
