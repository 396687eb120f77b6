set -o pipefail
timeout -k 10 60 ./tools/xorlane/xorlane && \
FMX_LIB=$PWD/form_amd/ab/libfmx_et.so timeout -k 10 120 python tools/extract_timing.py 2>&1 | grep -v amdgpu.ids | tail -3 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k extract -x -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -3
