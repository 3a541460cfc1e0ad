# Round-4: forward flux-pass ablations (state49)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
O=gpurun_out/r04
ABL_WORKLOAD=state49 timeout -k 10 300 python -u tools/ablate.py 0 11 12 14 15 16 > $O/abl2_state49_fwd.log 2>&1 || { cat $O/abl2_state49_fwd.log; exit 10; }
grep abl $O/abl2_state49_fwd.log
