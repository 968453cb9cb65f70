mkdir -p gpurun_out; : > gpurun_out/st.log
for gs in 1 8; do for reps in 1 8; do
  echo "=== gstride=$gs reps=$reps" >> gpurun_out/st.log
  WRNN_GSTRIDE=$gs WRNN_REPLICAS=$reps timeout -k 10 120 python tools/stamps.py quick >> gpurun_out/st.log 2>&1 || exit $?
done; done
