#!/bin/bash
# One GPU-box measurement pass (run via gpurun from the repo root). Each GPU step has its own
# time limit and the steps are chained: the first failure ends the script.
#   tools/gpu_measure.sh TAG [tests] [bench] [prof] [pmc] [aux]
set -e -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for what in "$@"; do
  case $what in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 120 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1 ;;
    bench)
      timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
        python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-aux > "$OUT/prof_bench.json" 2> "$OUT/prof.err" ;;
    pmc)
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-aux --kernel-timing-steps 0 > "$OUT/pmc_fetch.log" 2>&1
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-aux --kernel-timing-steps 0 > "$OUT/pmc_write.log" 2>&1 ;;
    pmcgemm)
      timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
        --output-format csv -d "$OUT/pmcgemm/p1" -o run -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-aux --kernel-timing-steps 0 > "$OUT/pmcgemm.log" 2>&1 ;;
    pmcmss2)
      bash tools/pmc_cmd.sh "$OUT/pmcmss2" bench_aux.py --workload mss --no-cpu-baseline --no-parity --steps 2 --warmup 1 ;;
    pmcall)  # FETCH / WRITE passes over the bench step and over each aux leg (traffic JSONs)
      for w in step frontend griffinlim mss; do
        if [ $w = step ]; then cmd="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-aux --kernel-timing-steps 0";
        else cmd="bench_aux.py --workload $w --no-cpu-baseline --no-parity --steps 2 --warmup 1"; fi
        for c in FETCH_SIZE WRITE_SIZE; do
          timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_${w}_$c" -o run -- \
            python3 $cmd > "$OUT/pmc_${w}_$c.log" 2>&1
        done
      done ;;
    pmcaux)
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcaux_fetch" -o run -- \
        python3 bench_aux.py --workload frontend --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/pmcaux_fetch.log" 2>&1
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmcaux_write" -o run -- \
        python3 bench_aux.py --workload frontend --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/pmcaux_write.log" 2>&1 ;;
    pmcgl)
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcgl_fetch" -o run -- \
        python3 bench_aux.py --workload griffinlim --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/pmcgl_fetch.log" 2>&1
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmcgl_write" -o run -- \
        python3 bench_aux.py --workload griffinlim --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/pmcgl_write.log" 2>&1 ;;
    pmcmss)
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcmss_fetch" -o run -- \
        python3 bench_aux.py --workload mss --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/pmcmss_fetch.log" 2>&1
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmcmss_write" -o run -- \
        python3 bench_aux.py --workload mss --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/pmcmss_write.log" 2>&1 ;;
    micro)
      make -C tools/micro > "$OUT/micro_build.log" 2>&1
      timeout -k 10 60 tools/micro/permlane_check > "$OUT/permlane_check.txt" 2>&1
      timeout -k 10 120 tools/micro/store_pattern > "$OUT/store_pattern.txt" 2>&1
      timeout -k 10 120 tools/micro/stft_stamps > "$OUT/stft_stamps.txt" 2>&1 ;;
    aux)
      timeout -k 10 400 python -u bench_aux.py > "$OUT/bench_aux.jsonl" 2> "$OUT/bench_aux.err" ;;
    layers)
      timeout -k 10 300 python -u tools/gemm_layers.py > "$OUT/gemm_layers.txt" 2> "$OUT/gemm_layers.err" ;;
    msstest)
      timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        -k "multiscale or mss" > "$OUT/pytest_mss.log" 2>&1 ;;
    gltest)
      timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        -k "griffinlim or istft or stft or mel" > "$OUT/pytest_gl.log" 2>&1 ;;
    auxgl)
      timeout -k 10 300 python -u bench_aux.py --workload griffinlim --no-cpu-baseline > "$OUT/aux_gl.json" 2> "$OUT/aux_gl.err" ;;
    auxmss)
      timeout -k 10 300 python -u bench_aux.py --workload mss --no-cpu-baseline > "$OUT/aux_mss.json" 2> "$OUT/aux_mss.err" ;;
    profaux)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profaux" -o run -- \
        python3 bench_aux.py --no-cpu-baseline --steps 5 --warmup 2 > "$OUT/profaux.json" 2> "$OUT/profaux.err" ;;
    msst)
      timeout -k 10 400 python -u -m pytest tests/test_gpu_spectral.py -x -v --timeout 120 --timeout-method thread \
        -k "multiscale or mss" > "$OUT/pytest_mss.log" 2>&1 ;;
    profmss)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profmss" -o run -- \
        python3 bench_aux.py --workload mss --no-cpu-baseline --no-parity --steps 5 --warmup 2 > "$OUT/profmss.json" 2> "$OUT/profmss.err" ;;
    gemmt)
      timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_bench_shapes.py -x -q \
        --timeout 120 --timeout-method thread > "$OUT/pytest_gemm.log" 2>&1 ;;
    pmcmsssq)
      timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv \
        -d "$OUT/pmcmss_sq" -o run -- python3 bench_aux.py --workload mss --no-cpu-baseline --no-parity \
        --steps 2 --warmup 1 > "$OUT/pmcmss_sq.log" 2>&1 ;;
    mssprobe)
      timeout -k 10 300 python -u tools/mss_probe.py > "$OUT/mss_probe.txt" 2>&1 ;;
    benchnoaux)
      timeout -k 10 300 python -u bench.py --no-aux > "$OUT/bench_noaux.json" 2> "$OUT/bench_noaux.err" ;;
    planes)
      make -C tools/micro gemm_planes > "$OUT/planes_build.log" 2>&1
      timeout -k 10 120 tools/micro/gemm_planes check > "$OUT/gemm_planes.txt" 2>&1 ;;
    rest)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_mss_train.py tests/test_gpu_spectral.py \
        tests/test_istft_grad.py tests/test_ops.py -m gpu -x -v -rP --timeout 120 --timeout-method thread \
        -k "B16 or mss or spectral or istft or opcheck or multiscale or stft or mel or griffin" > "$OUT/pytest_rest.log" 2>&1 ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    *) echo "unknown step $what"; exit 2 ;;
  esac
  echo "step $what ok"
done
