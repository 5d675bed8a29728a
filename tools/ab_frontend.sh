#!/bin/bash
# A/B of the config-2 front end (bench_aux frontend leg) between STFT kernel knobs, plus the
# STFT/mel parity tests. Dev tool, run on the GPU box:
#   tools/ab_frontend.sh OUTDIR [NAME=ENV ...]     e.g. base= lib2=MST_LIB_PATH=variants/x/libmst_hip.so
set -e -o pipefail
OUT=${1:?outdir}; shift; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_spectral.py tests/test_gpu_config2.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -k "stft or mel or dropin or logpow" > "$OUT/pytest_frontend.log" 2>&1
for rep in 1 2; do
  for v in "$@"; do
    name=${v%%=*}; envs=${v#*=}
    env $envs timeout -k 10 120 python bench_aux.py --workload frontend --no-cpu-baseline --steps 20 \
      > "$OUT/aux_${name}_$rep.jsonl" 2> "$OUT/aux_${name}_$rep.err"
  done
done
