set -o pipefail
# Round 3 evidence refresh after the Philox/CSR changes, part 2 first (the bench
# lines of part 1 read profiles/traffic_<config>.json): tools/gpu_profiles.sh,
# then single-stream (split1) CSR PMC passes of c2low and c2cli.
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_profiles.sh && \
CWQ_LIB_PATH=$PWD/tools/variants/libcwq_split1.so bash tools/gpu_pmc_csr.sh c2low r03_c2low_split1 && \
CWQ_LIB_PATH=$PWD/tools/variants/libcwq_split1.so bash tools/gpu_pmc_csr.sh c2cli r03_c2cli_split1 && \
echo r03p done
