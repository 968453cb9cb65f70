"""Sweep hand-off variants (replicas, polling waves) on the MoL B=1 loop; stamps per stage."""
import os
import sys
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
for reps in (8, 16):
    for pw in (2,):
        env = dict(os.environ, WRNN_REPLICAS=str(reps), WRNN_POLL_WAVES=str(pw))
        print(f"=== replicas={reps} poll_waves={pw}", flush=True)
        subprocess.run([sys.executable, os.path.join(HERE, "stamps.py"), "quick"], env=env, check=True)
