# GPU-box quick check used during development: parity tests, then the M1 / state49 bench lines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3
grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench.json").read().strip().splitlines()[-1])
print("state49", round(d["ms_per_step"], 3), "frac", round(d["roofline"]["frac"], 3))
for k, v in d.items():
    if isinstance(v, dict) and "bwd_ms" in v:
        print(k, {kk: round(vv, 3) for kk, vv in v.items() if kk.endswith("ms") or kk == "ms_per_step"})
PY
