for r in 1 2; do
  timeout -k 10 300 python tools/cpu_scaling.py 5 16 > gpurun_out/pin_$r.log 2>&1 || exit 1
  SG_CPU_NOPIN=1 timeout -k 10 300 python tools/cpu_scaling.py 5 16 > gpurun_out/nopin_$r.log 2>&1 || exit 1
done
for f in gpurun_out/pin_1.log gpurun_out/nopin_1.log gpurun_out/pin_2.log gpurun_out/nopin_2.log; do echo $f; tail -1 $f | cut -c1-260; done
