mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_chains.py tests/test_gpu_stream.py tests/test_gpu_multi.py tests/test_gpu_elementwise.py tests/test_gpu_nonfinite.py tests/test_gpu_fir.py tests/test_gpu_int8.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_sel.log; [ $rc = 0 ] || exit $rc
AB_WORK=fir,fm,am AB_ROUNDS=3 timeout -k 10 300 python tools/ab_time.py build/ab/libgsdr_r02base.so
