set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/gpu_suite_final.log 2>&1 && tail -1 gpurun_out/gpu_suite_final.log &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -1 &&
timeout -k 10 400 python -u bench.py --config c3 > gpurun_out/bench_c3_sh12.json 2> gpurun_out/bench_c3_sh12.err
