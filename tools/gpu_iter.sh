# GPU box, one development iteration: a pytest selection, bench lines, optional stage profile and
# rocprof kernel stats of one bench line.  Env: TESTS (pytest args), LINES (bench --lines), STAGE
# (stage_profile workload), KEXPR (pytest -k expression), PROF (bench line to profile with rocprofv3 --stats), TAG (file suffix).
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
T=${TAG:-iter}
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -k "${KEXPR:-}" -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_$T.log | tail -25
  [ $rc -ne 0 ] && { tail -40 gpurun_out/pytest_$T.log; exit $rc; }
fi
if [ -n "$LINES" ]; then
  timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --lines $LINES --no-cpu-baseline > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { tail -20 gpurun_out/bench_$T.err; exit 2; }
  python3 tools/bench_summary.py gpurun_out/bench_$T.json
fi
if [ -n "$STAGE" ]; then
  timeout -k 10 120 python -u tools/stage_profile.py $STAGE > gpurun_out/stage_${STAGE}_$T.txt 2>&1 || exit 4
  cat gpurun_out/stage_${STAGE}_$T.txt
fi
if [ -n "$PROF" ]; then
  cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kp -o kp -- python3 $R/bench.py --steps 3 --warmup 1 --lines $PROF --no-cpu-baseline > $R/gpurun_out/kp_$T.log 2>&1 || exit 3
  find /tmp/kp -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/kernel_stats_$T.csv \;
  head -14 $R/gpurun_out/kernel_stats_$T.csv | cut -c1-180
fi
exit 0
