# Round-4: last check of the committed binary: smoke and the -m gpu suite (without the full-size files)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
O=gpurun_out/r04
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_last.log 2>&1 || { cat $O/smoke_last.log; exit 20; }
tail -1 $O/smoke_last.log
timeout -k 10 560 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread --deselect tests/test_north_star.py --deselect tests/test_full_size.py > $O/pytest_last_gpu.log 2>&1
rc=$?
grep -E "^FAILED|passed|failed" $O/pytest_last_gpu.log | tail -8
exit $rc
