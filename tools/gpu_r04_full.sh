# Round-4: the full-size parity tests (numbers printed) + the new Bayes VAE / materialise tests, then
# small-model occupancy probes (N = 4096 vs 8192: one vs two tiles per CU).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
O=gpurun_out/r04
timeout -k 10 1000 python -u -m pytest tests/test_north_star.py tests/test_full_size.py tests/test_e2e_vae.py tests/test_materialize.py -v -s -m gpu --timeout 900 --timeout-method thread > $O/pytest_full3.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest_full3.log | tail -3
for wl in us_fp32 us_northstar; do
  for n in 4096 8192; do
    timeout -k 10 120 python -u bench.py --workload $wl --n-traj $n --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $O/probe_${wl}_${n}.json 2> $O/probe_${wl}_${n}.err || exit 30
  done
done
python3 - <<'PY'
import json
for wl in ("us_fp32", "us_northstar"):
    for n in (4096, 8192):
        d = json.load(open(f"gpurun_out/r04/probe_{wl}_{n}.json"))
        print(wl, n, "ms/step %.3f" % d["ms_per_step"], "fwd %.3f bwd %.3f" % (d["kernels"]["fwd_ms"], d["kernels"]["bwd_ms"]))
PY
exit $rc
