# decode_clock.py on each listed variant build (GPU box)
for k in ${VARIANTS:-base}; do
  echo "== $k"
  CWQ_LIB_PATH=$PWD/tools/vrun/libcwq_$k.so BATCHES=6 IDLE_S=0 timeout -k 10 120 python -u tools/decode_clock.py 2>&1 | grep -v amdgpu.ids || exit 1
done
