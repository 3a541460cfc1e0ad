# Round-4 final check of the committed tree: smoke(), the -m gpu suite, the full-size files, one bench line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
O=gpurun_out/r04
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_final4.log 2>&1 || { cat $O/smoke_final4.log; exit 20; }
tail -1 $O/smoke_final4.log
timeout -k 10 560 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread --deselect tests/test_north_star.py --deselect tests/test_full_size.py > $O/pytest_final4_gpu.log 2>&1
rc=$?
grep -E "^FAILED|passed|failed" $O/pytest_final4_gpu.log | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 560 python -u -m pytest tests/test_north_star.py tests/test_full_size.py -v -s -m gpu --timeout 520 --timeout-method thread > $O/pytest_final4_full.log 2>&1
rc2=$?
grep -E "^FAILED|passed|failed" $O/pytest_final4_full.log | tail -8
if [ $rc2 -ne 0 ]; then exit $rc2; fi
timeout -k 10 200 python -u bench.py --no-extra --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_final4.json 2> $O/bench_final4.err || { tail -5 $O/bench_final4.err; exit 21; }
cat $O/bench_final4.json
R=$(pwd)
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ks6 -o ks -- python3 $R/bench.py --no-extra --no-cpu-baseline --steps 5 --warmup 2 > $R/$O/ks6.log 2>&1 || exit 11
find /tmp/ks6 -name "*kernel_stats.csv" -exec cp {} $R/$O/state49_kernel_stats_final4.csv \;
cd $R
timeout -k 10 150 python -u tools/stage_profile.py state49 > $O/stage_final4_state49.txt 2>&1 || exit 9
grep -A9 "training forward" $O/stage_final4_state49.txt
