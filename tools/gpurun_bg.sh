# run a gpurun call in the background; its stdout/stderr go to $2 (default /tmp/w/gpu.txt)
/usr/local/graft/bin/gpurun --timeout ${3:-1200} -- "$1" > ${2:-/tmp/w/gpu.txt} 2>&1
echo "[exit $?]" >> ${2:-/tmp/w/gpu.txt}
