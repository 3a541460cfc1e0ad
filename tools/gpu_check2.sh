# GPU box: -m gpu suite, one step's device activities, the default bench line with selected extra lines
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/check}
LINES=${LINES:-state49_n2560_strong8_shard,north_star_M1,north_star_M1_fp32}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -v -s -m gpu --timeout 300 --timeout-method thread -x > $OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/pytest_gpu.log | tail -2
grep -E "^FAILED|Error" $OUT/pytest_gpu.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/step_ops.py > $OUT/step_ops.txt 2>&1 || exit 31
grep -E "device activities" $OUT/step_ops.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --lines $LINES --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit $?
python3 tools/bench_summary.py $OUT/bench.json
