# A/B of the in-tree library against _build/alt/libude_rk4.so (a dev build of a variant) on the
# default bench line, three alternating runs each.  Development only.
set -o pipefail
P=forecasting-influenza-using-universal-differential-equations_amd
L=$P/_build/libude_rk4.so
mkdir -p gpurun_out/ab_${WL:-state49}
cp $L gpurun_out/ab_${WL:-state49}/base.so.bin
for i in 1 2 3; do
  for v in base alt; do
    if [ $v = alt ]; then cp $P/_build/alt/libude_rk4.so $L; else cp gpurun_out/ab_${WL:-state49}/base.so.bin $L; fi
    timeout -k 10 120 python -u bench.py ${BENCH_ARGS:---no-extra} --no-cpu-baseline --workload ${WL:-state49} --steps ${STEPS:-20} --warmup 3 > gpurun_out/ab_${WL:-state49}/${v}_$i.json 2> gpurun_out/ab_${WL:-state49}/${v}_$i.err || { tail -5 gpurun_out/ab_${WL:-state49}/${v}_$i.err; exit 30; }
    echo "$v $i $(python3 tools/bench_summary.py gpurun_out/ab_${WL:-state49}/${v}_$i.json | tr "\n" " ")"
  done
done
cp gpurun_out/ab_${WL:-state49}/base.so.bin $L
rm -f gpurun_out/ab_${WL:-state49}/base.so.bin
