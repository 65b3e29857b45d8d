set -o pipefail
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -k "csr or uniform_odd or grouped or c2_image or ragged or pruned" > gpurun_out/t_csr.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c2cli --steps 3 --warmup 1 > gpurun_out/b_c2cli.log 2>&1 && \
CWQ_LIB_PATH=$PWD/tools/variants/libcwq_stats.so timeout -k 10 300 python -u tools/csr_stats.py c2cli > gpurun_out/csr_stats.log 2>&1
