#!/bin/bash
# round-4 batch u: upper bound of issuing the next span DMA before the FFT (variants/edma: the
# FFT scratch still overlaps the span, so its spectra are wrong: timing only,
# parity off).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4v; mkdir -p $O
b() { "$@" || { rc=$?; echo "stopping: rc=$rc"; exit $rc; }; }
for r in 1 2 3; do
  for lib in "" $PWD/variants/edma/libmst_hip.so; do
    echo "== lib ${lib:-in-tree}" >> $O/ab_fe.jsonl
    b env MST_LIB_PATH=$lib timeout -k 10 200 python -u bench_aux.py --workload frontend --no-cpu-baseline --no-parity --steps 20 --warmup 3 \
      >> $O/ab_fe.jsonl 2>> $O/ab_fe.err
  done
done
echo "all ok"
