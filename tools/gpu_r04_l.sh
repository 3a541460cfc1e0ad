# Round-4: forward tail-store batch A/B (state49, Bayes state49)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
O=gpurun_out/r04
for wl in state49 bayes_state49; do
  AB_WORKLOAD=$wl AB_VARIANTS="uc3:;uc5:-DUDE_TAIL_UC=5;uc9:-DUDE_TAIL_UC=9" AB_ROUNDS=4 timeout -k 10 400 python -u tools/ab_flags.py > $O/ab_uc_$wl.log 2>&1 || { cat $O/ab_uc_$wl.log; exit 11; }
  grep -v amdgpu.ids $O/ab_uc_$wl.log
done
