# Round-4: the -m gpu suite (without the full-size files), then the full-size files.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
O=gpurun_out/r04
timeout -k 10 560 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread --deselect tests/test_north_star.py --deselect tests/test_full_size.py > $O/pytest_h_gpu.log 2>&1
rc=$?
grep -E "^FAILED|passed|failed" $O/pytest_h_gpu.log | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 560 python -u -m pytest tests/test_north_star.py tests/test_full_size.py -v -s -m gpu --timeout 520 --timeout-method thread > $O/pytest_h_full.log 2>&1
rc2=$?
grep -E "^FAILED|passed|failed" $O/pytest_h_full.log | tail -8
exit $rc2
