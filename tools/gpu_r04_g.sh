# Round-4: checkpoint rows / latent rows A/B (state49, M1), forward stage profile, the -m gpu suite, then
# the full-size files.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
O=gpurun_out/r04
for wl in state49 us_northstar; do
  AB_WORKLOAD=$wl AB_VARIANTS="new:;c1l0:-DUDE_LAT_ROWS=0;old:-DUDE_LAT_ROWS=0 -DUDE_CKPT_ROWS=0" timeout -k 10 400 python -u tools/ab_flags.py > $O/ab_ck_$wl.log 2>&1 || { cat $O/ab_ck_$wl.log; exit 11; }
  grep -v amdgpu.ids $O/ab_ck_$wl.log
done
timeout -k 10 150 python -u tools/stage_profile.py state49 > $O/stage4_state49.txt 2>&1 || { cat $O/stage4_state49.txt; exit 9; }
grep -A9 "training forward" $O/stage4_state49.txt
timeout -k 10 560 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread --deselect tests/test_north_star.py --deselect tests/test_full_size.py > $O/pytest_g_gpu.log 2>&1
rc=$?
grep -E "^FAILED|passed|failed" $O/pytest_g_gpu.log | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 560 python -u -m pytest tests/test_north_star.py tests/test_full_size.py -v -s -m gpu --timeout 520 --timeout-method thread > $O/pytest_g_full.log 2>&1
rc2=$?
grep -E "^FAILED|passed|failed" $O/pytest_g_full.log | tail -8
exit $rc2
