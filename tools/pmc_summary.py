"""Summarise the FETCH_SIZE / WRITE_SIZE passes of tools/gpu_round.sh into profiles/<name>.json.

    python tools/pmc_summary.py gpurun_out profiles/r02_v5_pmc_traffic.json

Headline: per counter, the dispatch of the headline's persistent loop kernel (the longest
fatchord_xcd_kernel / fatchord_split_kernel / fatchord_loop_kernel dispatch in that pass), its
value (KiB per dispatch, as rocprofv3 reports these derived counters) and duration.  Other
configs (present when the passes ran bench.py --other-configs 1): per loop kernel, the summed
KiB over all its dispatches and the loop steps those dispatches covered.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports exactly half the bytes of
a wide coalesced read (16 B per lane, global_load and buffer_load ... lds alike), WRITE_SIZE the
exact bytes of 16-B-per-lane stores.  The XCD kernels' HBM reads are all such reads (float4 loads
of the conditioning terms, the slab prologue), so `bytes` = 2 x FETCH + WRITE; bench.py reads
`bytes` as `roofline.traffic`.  The rows kernels add 4-byte flag and 8-byte granule polls
(uncalibrated widths) beside their 16-B tile LDS-DMA: their per-step figures are approximate."""
import csv
import re
import json
import sys

HEADLINE = ("fatchord_xcd_kernel", "fatchord_split_kernel", "fatchord_loop_kernel")
# loop kernel -> (config key in bench.py's other_configs, loop steps of its dispatches in one
# bench.py --pmc-child run: the headline, the fold-batched line, then every other config, each
# generated ONCE, no warm-up calls).  The headline is the FIRST headline-kernel dispatch; later
# fatchord_xcd_kernel dispatches are the 8-utterance line (config2_8_streams).  The FIRST one-quad
# many-row dispatch is the fold-batched line (10 folds, one launch, before the other configs);
# later ones are config2_32_streams.
FIRST_OF = {"fatchord_xcdm_kernel<1,": "fatchord_xcdm_kernel<1,#first"}
OTHER = {"fatchord_xcdm_kernel<1,#first": ("fold_batched", 12100),          # 10 folds: 1 quad per XCD
         "fatchord_xcdm_kernel<4,": ("config3_mol_fold_60s", 12100),       # 115 rows: 4 quads per XCD
         "fatchord_xcdm_kernel<1,": ("config2_32_streams", 110275),        # 32 rows: 1 quad per XCD
         "fatchord_xcds_kernel": ("config4_sparse896_8utt", 110275),
         "deepmind_rows_kernel": ("config5_deepmind_32utt", 16000),
         "deepmind_xcd_kernel": ("config5_deepmind_32utt", 16000),
         "fatchord_xcd_kernel": ("config2_8_streams", 110275)}


def rows(path):
    with open(path) as f:
        yield from csv.DictReader(f)


def _order(r):
    return int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)


def loop_dispatch(path):
    """(name, KiB, duration) of the headline launch: the first headline-kernel dispatch."""
    hits = [r for r in rows(path) if any(k in r["Kernel_Name"] for k in HEADLINE)]
    if not hits:
        return None
    r = min(hits, key=_order)
    return r["Kernel_Name"], float(r["Counter_Value"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), _order(r)


def other_sums(path, headline_id):
    out = {}
    seen = set()
    for r in sorted(rows(path), key=_order):
        name = r["Kernel_Name"]
        # the many-row kernel's RAW instantiations (<NQ, dbg, true>: bench.py's config-1 lines)
        # are not config 3's
        if "fatchord_xcdm_kernel" in name and re.search(r"fatchord_xcdm_kernel<\d+, \w+, true>", name):
            continue
        if _order(r) == headline_id:
            continue
        for k in OTHER:
            if k in name:
                if k in FIRST_OF and k not in seen:
                    seen.add(k)
                    k = FIRST_OF[k]
                out[k] = out.get(k, 0.0) + float(r["Counter_Value"])
                break
    return out


def summarise(src):
    """The two passes under <src>/pmc_FETCH_SIZE, <src>/pmc_WRITE_SIZE → the traffic record."""
    counters, others = {}, {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        path = f"{src}/pmc_{c}/pmc_counter_collection.csv"
        name, kib, dur, hid = loop_dispatch(path)
        counters[c] = {"kernel": name, "value_kib": kib, "duration_ns": dur}
        for k, v in other_sums(path, hid).items():
            others.setdefault(k, {})[c] = v
    headline_bytes = 1024.0 * (2.0 * counters["FETCH_SIZE"]["value_kib"] + counters["WRITE_SIZE"]["value_kib"])
    cfg = {}
    for k, v in others.items():
        if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
            key, steps = OTHER[k]
            b = 1024.0 * (2.0 * v["FETCH_SIZE"] + v["WRITE_SIZE"])
            cfg[key] = {"kernel": k.split("<")[0], "fetch_kib": v["FETCH_SIZE"], "write_kib": v["WRITE_SIZE"], "loop_steps": steps,
                        "bytes_per_step": b / steps}
    return {
        "workload": "MOL rnn512 B=1 5 s (110275 steps), one persistent launch",
        "counters": counters,
        "bytes": headline_bytes,
        "other_configs": cfg,
        "note": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of bench.py --pmc-child (every "
                "config once, no warm-up). Counter values in KiB per dispatch; bytes = 1024 x (2 x FETCH_SIZE + "
                "WRITE_SIZE), the gfx950 correction for 16-B-per-lane reads (MI355X_MICROARCH.md). The XCD kernels' "
                "hand-offs are plain stores and 16-byte sc1 polls served by the XCD's L2; their HBM traffic is the "
                "float4 reads of the conditioning terms (one row: 32 x 640 = 20 480 B per step) and the draws.",
    }


def main(src, dst):
    out = summarise(src)
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
