set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06y; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_colblocks.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 900 bash tools/ab_lib.sh r06y/ablib_nt sddmm-gpu_amd/lib_exp/libbsmr_amd.so "C2 C2 C2k32 C2k512" > $O/ablib.log 2>&1 || exit 2
cat gpurun_out/r06y/ablib_nt/summary.txt
