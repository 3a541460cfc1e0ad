# Round-4: early activation-row stores A/B (state49, bayes_state49), then the -m gpu suite without the
# full-size files, then the full-size Bayes state49 test.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
O=gpurun_out/r04
for wl in state49 us_northstar; do
  timeout -k 10 150 python -u tools/stage_profile.py $wl > $O/stage_$wl.txt 2>&1 || { cat $O/stage_$wl.txt; exit 9; }
  grep -v amdgpu.ids $O/stage_$wl.txt
done
for wl in state49 bayes_state49; do
  AB_WORKLOAD=$wl AB_VARIANTS="early1:;early0:-DUDE_FWD_EARLY_ST=0" timeout -k 10 300 python -u tools/ab_flags.py > $O/ab_early_$wl.log 2>&1 || { cat $O/ab_early_$wl.log; exit 11; }
  grep -v amdgpu.ids $O/ab_early_$wl.log
done
timeout -k 10 560 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread --deselect tests/test_north_star.py --deselect tests/test_full_size.py > $O/pytest_c_gpu.log 2>&1
rc=$?
grep -E "^FAILED|passed|failed" $O/pytest_c_gpu.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python -u -m pytest -v -s -m gpu --timeout 450 --timeout-method thread \
  "tests/test_full_size.py::test_bayes_state49_full_batch" > $O/pytest_c_full.log 2>&1
rc2=$?
grep -E "passed|failed|bayes_state49 full|the [0-9]+ as one|well-conditioned|slice" $O/pytest_c_full.log
exit $(( rc > rc2 ? rc : rc2 ))
