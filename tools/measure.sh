# Measurement set (GPU box): the default bench line (all extra lines + CPU baselines), rocprof
# kernel stats (state49, north-star M1, M1 Fp [32,32], Bayes state49), FETCH / WRITE PMC passes of the
# default line, stage breakdowns.  UDE_COMMIT tags the PMC summaries with the measured commit.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
OUT=${OUT:-gpurun_out/measure}
mkdir -p $OUT
O=$R/$OUT
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > $O/bench_full.json 2> $O/bench_full.err || { tail -20 $O/bench_full.err; exit 21; }
python3 tools/bench_summary.py $O/bench_full.json
B="python3 $R/bench.py --no-extra --no-cpu-baseline"
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ks1 -o ks -- $B --steps 5 --warmup 2 > $O/ks1.log 2>&1 || exit 11
find /tmp/ks1 -name "*kernel_stats.csv" -exec cp {} $O/state49_kernel_stats.csv \;
# the roofline line recomputed from a kernel trace of the same command over its timed calls
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt -o kt -- $B --steps 20 --warmup 5 > $O/bench_trace.json 2> $O/kt.log || exit 17
find /tmp/kt -name "*kernel_trace.csv" -exec cp {} $O/state49_kernel_trace.csv \;
python3 $R/tools/roofline_trace.py $O/state49_kernel_trace.csv $O/bench_trace.json ${UDE_COMMIT:-} > $O/roofline_rocprof_state49.json || exit 18
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ks2 -o ks -- $B --workload us_northstar --steps 5 --warmup 2 > $O/ks2.log 2>&1 || exit 12
find /tmp/ks2 -name "*kernel_stats.csv" -exec cp {} $O/m1_kernel_stats.csv \;
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ks3 -o ks -- $B --workload us_fp32 --steps 5 --warmup 2 > $O/ks3.log 2>&1 || exit 13
find /tmp/ks3 -name "*kernel_stats.csv" -exec cp {} $O/m1_fp32_kernel_stats.csv \;
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ks4 -o ks -- $B --workload bayes_state49 --steps 5 --warmup 2 > $O/ks4.log 2>&1 || exit 16
find /tmp/ks4 -name "*kernel_stats.csv" -exec cp {} $O/bayes49_kernel_stats.csv \;
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pf -o pf -- $B --steps 3 --warmup 1 > $O/pf.log 2>&1 || exit 14
mkdir -p $O/pmc_fetch $O/pmc_write
find /tmp/pf -name "*counter_collection.csv" -exec cp {} $O/pmc_fetch/ \;
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pw -o pw -- $B --steps 3 --warmup 1 > $O/pw.log 2>&1 || exit 15
find /tmp/pw -name "*counter_collection.csv" -exec cp {} $O/pmc_write/ \;
cd $R
UDE_ROOFLINE_JSON=$O/roofline_rocprof_state49.json python3 tools/pmc_summary.py $O/pmc_fetch $O/pmc_write state49 > $O/pmc_summary.txt 2>&1 || true
cp profiles/pmc_state49_*.json $O/ 2>/dev/null || true
timeout -k 10 120 python -u tools/stage_profile.py state49 > $O/stage_state49.txt 2>&1 || exit 23
timeout -k 10 120 python -u tools/stage_profile.py us_northstar > $O/stage_m1.txt 2>&1 || exit 24
timeout -k 10 120 python -u tools/stage_profile.py us_fp32 > $O/stage_m1_fp32.txt 2>&1 || exit 25
timeout -k 10 120 python -u tools/stage_profile.py bayes_state49 > $O/stage_bayes49.txt 2>&1 || exit 26
exit 0
