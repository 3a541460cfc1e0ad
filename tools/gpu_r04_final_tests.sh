# Round-4 GPU check: the full-size parity tests first (printing their numbers), then the rest of
# the -m gpu suite.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
O=gpurun_out/r04
timeout -k 10 560 python -u -m pytest tests/test_north_star.py tests/test_full_size.py -v -s -m gpu --timeout 520 --timeout-method thread > $O/pytest_final_full.log 2>&1
rc1=$?
grep -E "passed|failed" $O/pytest_final_full.log | tail -3
if [ $rc1 -ne 0 ] && [ $rc1 -ne 1 ]; then exit $rc1; fi
timeout -k 10 560 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread --deselect tests/test_north_star.py --deselect tests/test_full_size.py > $O/pytest_final_gpu.log 2>&1
rc2=$?
grep -E "passed|failed" $O/pytest_final_gpu.log | tail -3
exit $(( rc1 > rc2 ? rc1 : rc2 ))
