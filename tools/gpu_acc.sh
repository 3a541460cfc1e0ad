# GPU box: per-trajectory accuracy diagnostic, one step's kernels, a quick bench, the full-size parity tests
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/acc}
mkdir -p $OUT
timeout -k 10 300 python -u tools/ns_traj.py 2994 3613 516 3746 3297 100 > $OUT/ns_traj.txt 2>&1 || exit 41
timeout -k 10 200 python -u tools/step_ops.py > $OUT/step_ops.txt 2>&1 || exit 42
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --lines state49_n2560_strong8_shard,north_star_M1 \
  --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 43
timeout -k 10 1200 python -u -m pytest tests/test_full_size.py tests/test_north_star.py -v -s -m gpu --timeout 1100 \
  --timeout-method thread > $OUT/pytest_full.log 2>&1
grep -E "passed|failed" $OUT/pytest_full.log | tail -2
