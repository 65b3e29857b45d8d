set -o pipefail
for c in pln c2cli; do
  echo "## $c"
  BENCH_ARGS="--config $c" bash tools/variants.sh run
done > gpurun_out/var_csr.log 2>&1
