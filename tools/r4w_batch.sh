#!/bin/bash
# round-4 batch w (final build): three default bench lines back to back (run-to-run spread on one
# box) and the rocprof stats of bench_aux's spectral legs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4w; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py >> $O/bench_repeat.jsonl 2>> $O/bench_repeat.err || exit $?
done
bash tools/gpu_measure.sh r4w profaux
