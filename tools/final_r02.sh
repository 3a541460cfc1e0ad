# Round-end measurement set (GPU box): parity tests, full bench line, stage breakdowns,
# rocprof kernel stats and FETCH/WRITE PMC passes (tools/prof_r02.sh).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 20
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || exit 21
timeout -k 10 120 python -u tools/stage_profile.py us_northstar > gpurun_out/stage_m1.txt 2>&1 || exit 22
timeout -k 10 120 python -u tools/stage_profile.py state49 > gpurun_out/stage_s49.txt 2>&1 || exit 23
bash tools/prof_r02.sh || exit $?
exit 0
