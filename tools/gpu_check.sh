# GPU-box check used during development: parity tests, bench line, M1 stage profile + rocprof.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3
grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
tail -c 1500 gpurun_out/bench.json
if [ "$1" = "prof" ]; then
  timeout -k 10 120 python -u tools/stage_profile.py us_northstar > gpurun_out/stage_m1.txt 2>&1 || exit $?
  cat gpurun_out/stage_m1.txt
  timeout -k 10 120 python -u tools/stage_profile.py state49 > gpurun_out/stage_s49.txt 2>&1 || exit $?
  cat gpurun_out/stage_s49.txt
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_m1 -o m1 -- python3 bench.py --workload us_northstar --steps 5 --warmup 2 --no-extra --no-cpu-baseline > gpurun_out/prof_m1.log 2>&1 || exit $?
  find /tmp/prof_m1 -name "*kernel_stats.csv" -exec cp {} gpurun_out/m1_kernel_stats.csv \;
fi
exit $rc
