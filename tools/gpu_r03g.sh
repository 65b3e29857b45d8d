set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 && tail -1 gpurun_out/t_all.log && \
C3_SPLIT=1 C3_NO_CPROFILE=1 timeout -k 10 120 python -u tools/c3_pyprof.py > gpurun_out/c3_k.log 2>&1 && grep 'ms per call' gpurun_out/c3_k.log && \
C3_CALLS=5 C3_NO_CPROFILE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3tl -o run --output-format csv -- python3 tools/c3_pyprof.py > gpurun_out/c3_tl.log 2>&1 && \
python tools/timeline.py gpurun_out/prof_c3tl 6 > gpurun_out/c3_timeline.txt && grep -c small_surv gpurun_out/c3_timeline.txt


timeout -k 10 120 python -u tools/c3_pyparts.py > gpurun_out/c3_pyparts.log 2>&1; tail -2 gpurun_out/c3_pyparts.log
VARIANTS="base dnt base dnt" bash tools/decode_variants.sh > gpurun_out/decode_var.log 2>&1; cat gpurun_out/decode_var.log
