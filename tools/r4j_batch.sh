#!/bin/bash
# round-4 final-tree validation: every GPU test (a test failure is recorded and the batch goes on;
# a crash or timeout ends it), smoke, the default bench line, its rocprof stats, and the STFT
# traffic passes of the shipped build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_measure.sh r4j smoke bench prof pmcaux
