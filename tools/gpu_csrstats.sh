set -o pipefail
for c in c2low c2cli; do
  CWQ_LIB_PATH=$PWD/tools/variants/libcwq_stats.so timeout -k 10 300 python -u tools/csr_stats.py $c >> gpurun_out/csrstats.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --config $c --steps 2 --warmup 1 >> gpurun_out/csrstats.log 2>&1 || exit 1
done
