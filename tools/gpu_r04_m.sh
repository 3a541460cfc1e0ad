# Round-4: fp32 stage sums of the forward side statistics A/B (state49), then smoke, the -m gpu suite,
# the full-size files and one bench line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
O=gpurun_out/r04
AB_WORKLOAD=state49 AB_VARIANTS="s32:;s64:-DUDE_STAT32=0" AB_ROUNDS=4 timeout -k 10 300 python -u tools/ab_flags.py > $O/ab_stat32_state49.log 2>&1 || { cat $O/ab_stat32_state49.log; exit 11; }
grep -v amdgpu.ids $O/ab_stat32_state49.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_m.log 2>&1 || { cat $O/smoke_m.log; exit 20; }
tail -1 $O/smoke_m.log
timeout -k 10 560 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread --deselect tests/test_north_star.py --deselect tests/test_full_size.py > $O/pytest_m_gpu.log 2>&1
rc=$?
grep -E "^FAILED|passed|failed" $O/pytest_m_gpu.log | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 560 python -u -m pytest tests/test_north_star.py tests/test_full_size.py -v -s -m gpu --timeout 520 --timeout-method thread > $O/pytest_m_full.log 2>&1
rc2=$?
grep -E "^FAILED|passed|failed" $O/pytest_m_full.log | tail -8
if [ $rc2 -ne 0 ]; then exit $rc2; fi
timeout -k 10 200 python -u bench.py --no-extra --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_m.json 2> $O/bench_m.err || { tail -5 $O/bench_m.err; exit 21; }
cat $O/bench_m.json
