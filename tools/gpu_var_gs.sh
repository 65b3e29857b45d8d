set -o pipefail
echo "## c2cli" > gpurun_out/var_gs.log
for k in base gs16 gs64 gs16n; do
  echo "== $k" >> gpurun_out/var_gs.log
  CWQ_LIB_PATH=$PWD/tools/variants/libcwq_$k.so timeout -k 10 300 python -u bench.py --config c2cli --steps 3 --warmup 1 >> gpurun_out/var_gs.log 2>&1 || exit 1
done
