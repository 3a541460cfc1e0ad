# Round-4: re-run the fixed full-size / e2e tests, then a per-kernel trace of the default bench step.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out/r04
O=$R/gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests/test_north_star.py tests/test_full_size.py tests/test_e2e_vae.py tests/test_materialize.py -v -s -m gpu --timeout 800 --timeout-method thread -k "m1_full_size or bayes_state49 or us_bayes or test_vae_step_fused or store_released or materialized_lists_bayes" > $O/pytest_full4.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest_full4.log | tail -3
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ks1 -o ks -- python3 $R/bench.py --no-extra --no-cpu-baseline --steps 5 --warmup 2 > $O/ks_state49.log 2>&1 || exit 11
find /tmp/ks1 -name "*kernel_stats.csv" -exec cp {} $O/state49_kernel_stats.csv \;
find /tmp/ks1 -name "*kernel_trace.csv" -exec cp {} $O/state49_kernel_trace.csv \;
cd $R
# stored activations (default) vs the Recompute<M> view (forced by a 1-byte activation budget)
timeout -k 10 200 python -u bench.py --no-extra --no-cpu-baseline --steps 10 --warmup 3 > $O/ab_store.json 2>/dev/null || exit 13
UDE_ACT_BUDGET_BYTES=1 timeout -k 10 200 python -u bench.py --no-extra --no-cpu-baseline --steps 10 --warmup 3 > $O/ab_recompute.json 2>/dev/null || exit 14
python3 -c "
import json
for n in ('ab_store', 'ab_recompute'):
    d = json.load(open('gpurun_out/r04/%s.json' % n)); print(n, 'ms/step %.3f fwd %.3f bwd %.3f' % (d['ms_per_step'], d['kernels']['fwd_ms'], d['kernels']['bwd_ms']))
"
timeout -k 10 300 python -u tools/ab_gst_r1.py > $O/ab_gst_r1.log 2>&1 || exit 12
cat $O/ab_gst_r1.log
exit $rc
