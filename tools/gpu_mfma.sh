mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fir.py -q -x -k "mfma or variants" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_mfma.log 2>&1; rc=$?; tail -5 gpurun_out/t_mfma.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python tools/mfma_bits.py 2>&1 | grep -v amdgpu.ids || exit 1
bash tools/power_split.sh ${VARIANTS:-0 13 104 113}
