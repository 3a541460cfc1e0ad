# GPU box: Bayes parity tests (whole-solve GST path), Bayes bench lines, rocprof kernel stats of bayes_state49
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_bayes.py -x -v --timeout 300 --timeout-method thread -k "${KSEL:-.}" > gpurun_out/pytest_bayes.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_bayes.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --lines ${LINES:-bayes_state49,bayes_M1} --no-cpu-baseline > gpurun_out/bench_bayes.json 2> gpurun_out/bench_bayes.err || exit 2
python3 tools/bench_summary.py gpurun_out/bench_bayes.json
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kb -o kb -- python3 $R/bench.py --steps 3 --warmup 1 --lines bayes_state49 --no-cpu-baseline > $R/gpurun_out/kb.log 2>&1 || exit 3
find /tmp/kb -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/bayes49_kernel_stats.csv \;
head -12 $R/gpurun_out/bayes49_kernel_stats.csv | cut -c1-200
if [ -n "$STAGE" ]; then
  cd $R && timeout -k 10 120 python -u tools/stage_profile.py $STAGE > gpurun_out/stage_$STAGE.txt 2>&1 || exit 4
  cat gpurun_out/stage_$STAGE.txt
fi
