mkdir -p gpurun_out
timeout -k 10 300 python tools/diag_loop.py > gpurun_out/diag.log 2>&1 || exit $?
timeout -k 10 120 python tools/stamps.py quick > gpurun_out/st.log 2>&1
