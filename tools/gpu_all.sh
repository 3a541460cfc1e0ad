# GPU box: full -m gpu suite then the default bench line (with its extra lines)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -v -s -m gpu --timeout 900 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -2
grep -E "^FAILED|north-star|VJP on|whole-batch|dopri5 full|e2e worst" gpurun_out/pytest_gpu.log | head -30
[ $rc -ne 0 ] && [ "${CONTINUE_ON_FAIL:-0}" != "1" ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
python3 tools/bench_summary.py gpurun_out/bench.json
