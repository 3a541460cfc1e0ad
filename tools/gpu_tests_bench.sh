# GPU box: the -m gpu suite, then the default bench line without extra lines (quick check of a tree)
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/check}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -v -s -m gpu --timeout 300 --timeout-method thread -x > $OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/pytest_gpu.log | tail -2
grep -E "^FAILED|Error" $OUT/pytest_gpu.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit $?
python3 tools/bench_summary.py $OUT/bench.json
