set -e
timeout -k 10 400 python -m pytest tests/test_gpu_chains.py tests/test_gpu_fir.py -q -x -p no:cacheprovider 2>&1 | tail -3
timeout -k 10 200 python tools/fm_probe.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python tools/fm_probe.py --mode am 2>&1 | grep -v amdgpu.ids
