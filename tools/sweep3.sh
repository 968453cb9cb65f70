mkdir -p gpurun_out
rocprofv3 -L > gpurun_out/counters.txt 2>&1
timeout -k 10 120 python tools/stamps.py quick > gpurun_out/st.log 2>&1
