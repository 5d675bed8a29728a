set -e
mkdir -p gpurun_out/r02_abl
for v in ${ABL_VARIANTS:-base NOFFT NOLOG NOWRITE}; do
  if [ $v = base ]; then unset MST_LIB_PATH; else export MST_LIB_PATH=$PWD/variants/abl_$v/libmst_hip.so; fi
  timeout -k 10 120 python -u bench_aux.py --workload frontend --no-cpu-baseline > gpurun_out/r02_abl/$v.jsonl 2> gpurun_out/r02_abl/$v.err
done
