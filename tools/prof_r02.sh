export TMPDIR=/tmp
B="python3 bench.py --no-extra --no-cpu-baseline"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ks1 -o ks -- $B --steps 5 --warmup 2 > gpurun_out/ks1.log 2>&1 || exit 11
find /tmp/ks1 -name "*kernel_stats.csv" -exec cp {} gpurun_out/state49_kernel_stats.csv \;
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ks2 -o ks -- $B --workload us_northstar --steps 5 --warmup 2 > gpurun_out/ks2.log 2>&1 || exit 12
find /tmp/ks2 -name "*kernel_stats.csv" -exec cp {} gpurun_out/m1_kernel_stats.csv \;
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pf -o pf -- $B --steps 3 --warmup 1 > gpurun_out/pf.log 2>&1 || exit 13
mkdir -p gpurun_out/pmc_fetch gpurun_out/pmc_write
find /tmp/pf -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc_fetch/ \;
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pw -o pw -- $B --steps 3 --warmup 1 > gpurun_out/pw.log 2>&1 || exit 14
find /tmp/pw -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc_write/ \;
ls -la gpurun_out/pmc_fetch gpurun_out/pmc_write
