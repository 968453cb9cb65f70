#!/bin/bash
# ISA of one kernel source exactly as wavernn_amd/build.py compiles it (its flags + -S), for
# reading the compiled critical paths:  tools/isa.sh fatchord_xcd.hip /tmp/xcd.s
set -e
src=$1; out=${2:-/tmp/$(basename $src .hip).s}
R=$(cd "$(dirname "$0")/.." && pwd)
python3 - "$R" "$src" "$out" <<'PY'
import sys, subprocess, os
R, src, out = sys.argv[1:4]
sys.path.insert(0, R)
from wavernn_amd import build as b
full = os.path.join(R, "wavernn_amd", "csrc", src)
cmd = b._compile_cmd(full)
# replace the output object with assembly
i = cmd.index("-o")
cmd = cmd[:i] + ["-S", "--cuda-device-only", "-o", out] + cmd[i + 2:]
cmd = [c for c in cmd if c != "-c"]
subprocess.run(cmd, check=True)
PY
echo "$out"
