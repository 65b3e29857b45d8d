set -o pipefail
echo "## importance" > gpurun_out/var_imp.log
CWQ_LIB_PATH=$PWD/tools/variants/libcwq_idyn.so timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "importance" >> gpurun_out/var_imp.log 2>&1 || exit 1
for c in i1 i2; do
for k in base idyn; do
  echo "== $c $k" >> gpurun_out/var_imp.log
  CWQ_LIB_PATH=$PWD/tools/variants/libcwq_$k.so timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 >> gpurun_out/var_imp.log 2>&1 || exit 1
done
done
