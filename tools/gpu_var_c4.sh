set -o pipefail
echo "## c4" > gpurun_out/var_c4.log
for k in base mask7 mask31 cap512 w7; do
  echo "== $k" >> gpurun_out/var_c4.log
  CWQ_LIB_PATH=$PWD/tools/variants/libcwq_$k.so timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --steps 3 --warmup 1 >> gpurun_out/var_c4.log 2>&1 || exit 1
done
