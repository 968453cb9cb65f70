set -e
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag_loop.py > gpurun_out/diag.log 2>&1
for dp in 0 1; do
  echo "=== delay_poll=$dp" >> gpurun_out/st.log
  WRNN_DELAY_POLL=$dp timeout -k 10 120 python tools/stamps.py quick >> gpurun_out/st.log 2>&1
done
