# Round-4: Bayes backward glue (one fused d std, row-vectorized static-dim time sums): Bayes bench lines,
# the -m gpu suite and the full-size files.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
O=gpurun_out/r04
timeout -k 10 300 python -u bench.py --no-cpu-baseline --lines bayes_M1,bayes_state49 --steps 10 --warmup 3 > $O/bench_bayes_k.json 2> $O/bench_bayes_k.err || { tail -5 $O/bench_bayes_k.err; exit 21; }
python3 -c "
import json; d=json.load(open('$O/bench_bayes_k.json')); print({k: d[k] for k in ('bayes_M1', 'bayes_state49') if k in d})"
timeout -k 10 560 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread --deselect tests/test_north_star.py --deselect tests/test_full_size.py > $O/pytest_k_gpu.log 2>&1
rc=$?
grep -E "^FAILED|passed|failed" $O/pytest_k_gpu.log | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 560 python -u -m pytest tests/test_north_star.py tests/test_full_size.py -v -s -m gpu --timeout 520 --timeout-method thread > $O/pytest_k_full.log 2>&1
rc2=$?
grep -E "^FAILED|passed|failed" $O/pytest_k_full.log | tail -8
exit $rc2
