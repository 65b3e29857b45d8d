set -o pipefail
echo "## c2cli" > gpurun_out/var_tile.log
for k in base t512 t256b t2048; do
  echo "== $k" >> gpurun_out/var_tile.log
  CWQ_LIB_PATH=$PWD/tools/variants/libcwq_$k.so timeout -k 10 300 python -u bench.py --config c2cli --steps 3 --warmup 1 >> gpurun_out/var_tile.log 2>&1 || exit 1
done
