# run a gpurun call in the background; its stdout/stderr go to $2 (default /tmp/w/gpu.txt).
# Re-submits only when gpurun answers 3 (no box / slot free: nothing ran, nothing charged).
out=${2:-/tmp/w/gpu.txt}
: > $out
for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
  /usr/local/graft/bin/gpurun --timeout ${3:-1200} -- "$1" >> $out 2>&1
  rc=$?
  echo "[exit $rc]" >> $out
  [ $rc -ne 3 ] && break
  sleep 100
done
