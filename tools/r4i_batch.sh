#!/bin/bash
# round-4 batch i: FMA-form FFT butterflies (variants/fma) vs the in-tree build on the spectral
# legs; SQ counters on the STFT for both; STFT traffic on the variant.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4i; mkdir -p $O
V=$PWD/variants/fma/libmst_hip.so
t() { local log=$1; shift; "$@" > "$O/$log" 2>&1; local rc=$?; echo "$log rc=$rc";
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $log rc=$rc"; exit $rc; fi; }
b() { "$@" || { rc=$?; echo "stopping: rc=$rc"; exit $rc; }; }
PT="python -u -m pytest -q --timeout 120 --timeout-method thread"
t pytest_fma.log env MST_LIB_PATH=$V timeout -k 10 500 $PT tests/test_gpu_spectral.py tests/test_gpu_config2.py tests/test_istft_grad.py -m gpu
for r in 1 2 3; do
  for lib in "" $V; do
    for w in frontend griffinlim mss; do
      echo "== lib ${lib:-in-tree} $w" >> $O/ab_aux.jsonl
      b env MST_LIB_PATH=$lib timeout -k 10 200 python -u bench_aux.py --workload $w --no-cpu-baseline --steps 20 --warmup 3 \
        >> $O/ab_aux.jsonl 2>> $O/ab_aux.err
    done
  done
done
echo "ab ok"
b bash tools/pmc_cmd.sh $O/pmc_stft_tree bench_aux.py --workload frontend --no-cpu-baseline --no-parity --steps 2 --warmup 1
b env MST_LIB_PATH=$V bash tools/pmc_cmd.sh $O/pmc_stft_fma bench_aux.py --workload frontend --no-cpu-baseline --no-parity --steps 2 --warmup 1
b env MST_LIB_PATH=$V bash tools/gpu_measure.sh r4i pmcaux
echo "all ok"
