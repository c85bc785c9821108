"""Summarise tools/pmc_probe.py counter passes: per workload and counter, the mean per dispatch
of the probed kernel (k_stream_read / k_fedavg_pipe), plus the kernel duration.

Usage: python tools/pmc_probe_report.py gpurun_out/<tag>/pmcprobe
(expects <dir>/<workload>_<pass>/run_counter_collection.csv)
"""
import csv
import glob
import json
import os
import sys


def main(d):
    res = {}
    for path in sorted(glob.glob(os.path.join(d, "*", "run_counter_collection.csv"))):
        wl = os.path.basename(os.path.dirname(path)).rsplit("_", 1)[0]
        rows = [r for r in csv.DictReader(open(path))
                if "k_stream_read" in r["Kernel_Name"] or "k_fedavg_pipe" in r["Kernel_Name"]]
        acc = {}
        for r in rows:
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        ent = res.setdefault(wl, {})
        for k, v in acc.items():
            ent[k] = sum(v) / len(v)
        tr = os.path.join(os.path.dirname(path), "run_kernel_trace.csv")
        if os.path.exists(tr):
            ds = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(tr))
                  if "k_stream_read" in r["Kernel_Name"] or "k_fedavg_pipe" in r["Kernel_Name"]]
            if ds:
                ent.setdefault("dur_ms", []).append(sum(ds) / len(ds) / 1e6)
    for wl, ent in res.items():
        print(json.dumps({"workload": wl, **ent}))


if __name__ == "__main__":
    main(sys.argv[1])
