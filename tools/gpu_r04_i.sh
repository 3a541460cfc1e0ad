# Round-4: backward ablations (state49): partner dW MFMAs, activation-row DMA, critical input-gradient phases
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
O=gpurun_out/r04
ABL_WORKLOAD=state49 timeout -k 10 300 python -u tools/ablate.py 0 7 21 22 > $O/abl3_state49_bwd.log 2>&1 || { cat $O/abl3_state49_bwd.log; exit 10; }
grep abl $O/abl3_state49_bwd.log
