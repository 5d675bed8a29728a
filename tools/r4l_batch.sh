#!/bin/bash
# round-4 final tree (after the InstanceNorm pair accesses): every GPU test, smoke, the default
# bench line with its aux legs, rocprof stats.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4l; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_measure.sh r4l smoke bench prof
