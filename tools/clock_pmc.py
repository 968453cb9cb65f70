"""Effective clock of each dispatch from a rocprofv3 GRBM_GUI_ACTIVE pass
(MI355X_MICROARCH.md 'DVFS give-back': cycles summed over the 8 XCDs / 8 / wall time).
    python tools/clock_pmc.py gpurun_out/clk/pmc_counter_collection.csv [substr]"""
import csv
import sys


def main(path, sub=""):
    for r in csv.DictReader(open(path)):
        if sub not in r["Kernel_Name"] or r["Counter_Name"] != "GRBM_GUI_ACTIVE":
            continue
        ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        cyc = float(r["Counter_Value"])
        print(f"{r['Kernel_Name'][:60]:60s} grid {r.get('Grid_Size', '?'):>8s} {ns / 1e6:9.3f} ms  "
              f"sum/8/t {cyc / 8 / ns * 1e3:7.1f} MHz  sum/t {cyc / ns * 1e3:8.1f} MHz", flush=True)


if __name__ == "__main__":
    main(*sys.argv[1:])
