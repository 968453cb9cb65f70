"""Summarise the FETCH_SIZE / WRITE_SIZE passes of tools/gpu_round.sh into profiles/<name>.json.

    python tools/pmc_summary.py gpurun_out profiles/r01_v4_pmc_traffic.json

Takes, per counter, the dispatch of the headline's persistent loop kernel (the longest
fatchord_xcd_kernel / fatchord_split_kernel / fatchord_loop_kernel dispatch in that pass) and stores its value (KiB per dispatch, as rocprofv3 reports these
derived counters) and duration; bench.py reads the sum as `roofline.traffic`."""
import csv
import json
import sys


def loop_dispatch(path):
    best = None
    with open(path) as f:
        for r in csv.DictReader(f):
            if not any(k in r["Kernel_Name"] for k in ("fatchord_xcd_kernel", "fatchord_split_kernel", "fatchord_loop_kernel")):
                continue
            dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            if best is None or dur > best[2]:
                best = (r["Kernel_Name"], float(r["Counter_Value"]), dur)
    return best


def main(src, dst):
    counters = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        name, kib, dur = loop_dispatch(f"{src}/pmc_{c}/pmc_counter_collection.csv")
        counters[c] = {"kernel": name, "value_kib": kib, "duration_ns": dur}
    out = {
        "workload": "MOL rnn512 B=1 5 s (110275 steps), one persistent launch",
        "counters": counters,
        "note": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (bench.py --steps 1). "
                "Units KiB per dispatch (no width correction applied: the XCD kernel's hand-offs are plain "
                "8-byte stores and 16-byte sc1 polls served by the XCD's L2, its HBM traffic is the 16-byte "
                "reads of the 640 B/step/workgroup conditioning terms).",
    }
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
