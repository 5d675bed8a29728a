#!/bin/bash
# Same-box A/B of the multi-scale loss workload (dev tool; via gpurun from the repo root): the
# spectral GPU tests on the in-tree build, then bench_aux.py --workload mss alternating the in-tree
# library with VAR (default variants/base/libmst_hip.so), N rounds.
#   tools/ab_mss.sh TAG [tests-selection] ; env: VAR, ROUNDS (3)
set -e -o pipefail
OUT=gpurun_out/${1:?tag}; mkdir -p "$OUT"
V=${VAR:-variants/base/libmst_hip.so}
export TMPDIR=/tmp
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest $2 -x -v --timeout 120 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1
  echo "tests ok"
fi
for r in $(seq 1 ${ROUNDS:-3}); do
  for lib in "" $V; do
    echo "== lib ${lib:-in-tree}" >> "$OUT/ab_mss.jsonl"
    MST_LIB_PATH=$lib timeout -k 10 200 python -u bench_aux.py --workload mss --no-cpu-baseline \
      >> "$OUT/ab_mss.jsonl" 2>> "$OUT/ab_mss.err"
  done
done
echo "bench ok"
