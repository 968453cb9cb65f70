"""Build an alternative library for A/B timing (tools/ab_libs.sh): the in-tree objects, with
named sources (comma-separated) recompiled under extra flags, linked to tools/_alt/<name>.so.
    python tools/build_alt.py <name> <source.hip>[,<source2>] [-DFLAG=V ...]"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wavernn_amd import build as hb  # noqa: E402


def main(name, src, *flags):
    hb.build(verbose=False)
    objdir = os.path.join(os.path.dirname(hb.OUT), "obj")
    alt = os.path.join(hb.REPO, "tools", "_alt")
    os.makedirs(alt, exist_ok=True)
    objs = []
    for s in hb.SOURCES:
        base = os.path.basename(s)
        obj = os.path.join(objdir, base + ".o")
        if base in src.split(","):
            obj = os.path.join(alt, f"{name}_{base}.o")
            cmd = [hb.hipcc(), f"--offload-arch={hb.ARCH}", "-O3", "-std=c++17", "-fPIC",
                   "-I" + os.path.join(hb.REPO, "include"), *hb.EXTRA_FLAGS.get(base, []), *flags, "-c", s, "-o", obj]
            subprocess.run(cmd, check=True)
        objs.append(obj)
    out = os.path.join(alt, name + ".so")
    subprocess.run([hb.hipcc(), f"--offload-arch={hb.ARCH}", "-shared", "-fPIC", *objs, "-lrocblas", "-o", out], check=True)
    print(out)


if __name__ == "__main__":
    main(*sys.argv[1:])
