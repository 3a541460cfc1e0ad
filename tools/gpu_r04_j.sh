# Round-4: critical-path issue priority A/B (state49, M1, M1 Fp[32,32])
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
O=gpurun_out/r04
for wl in state49 us_northstar us_fp32; do
  AB_WORKLOAD=$wl AB_VARIANTS="prio1:;prio0:-DUDE_PRIO=0" timeout -k 10 300 python -u tools/ab_flags.py > $O/ab_prio_$wl.log 2>&1 || { cat $O/ab_prio_$wl.log; exit 11; }
  grep -v amdgpu.ids $O/ab_prio_$wl.log
done
