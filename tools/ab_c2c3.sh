set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
for v in main old; do
  lp=$PWD/compression_without_quantization_amd/libcwq.so; [ $v = old ] && lp=$PWD/tools/vrun/libcwq_old.so
  for c in c2 c3; do
    CWQ_LIB_PATH=$lp timeout -k 10 300 python -u bench.py --config $c --no-cpu --no-e2e --steps 20 --warmup 3 > gpurun_out/ab_${v}_${c}_$r.log 2>&1 || exit 1
    python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/ab_${v}_${c}_$r.log') if l.startswith('{')][-1]; print('$v $c', round(d['value'],1), round(d['ms_per_step'],3), d['roofline']['kernel_ms'])"
  done
done
done
