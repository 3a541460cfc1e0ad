export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_loss_head.py tests/test_e2e_vae.py > gpurun_out/pt_lh.log 2>&1; rc=$?; tail -3 gpurun_out/pt_lh.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lh -o lh -- python3 tools/loss_head_timing.py > gpurun_out/lh.log 2>&1 || exit 5
find /tmp/lh -name "*kernel_stats.csv" -exec cp {} gpurun_out/lh_kernel_stats.csv \;
grep -v "^[WE]20" gpurun_out/lh.log | tail -3
