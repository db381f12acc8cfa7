#!/usr/bin/env python3
"""Per-kernel means of a rocprofv3 --pmc pass with SQ_INSTS_VALU (and any
other counters) from counter_collection.csv, as the JSON bench.py reads for
its VALU-issue roofline (roofline_valu).  SQ_INSTS_VALU counts wave64 VALU
instructions over the whole chip; GRBM_GUI_ACTIVE is summed over the 8 XCDs.

    python tools/pmc_valu.py counter_collection.csv --workload 4096x4096 \
        --command "..." -o profiles/r2/pmc_valu_4096.json
"""
import argparse
import csv
import json
import re
from collections import defaultdict


def short(name):
    m = re.search(r"(k_\w+(<[^>]*>)?)", name)
    return m.group(1) if m else name.split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--command", default="")
    ap.add_argument("-o", required=True)
    ap.add_argument("--persist-blocks", type=int, default=0,
                    help="T-sweep blocks one k_jacobi_persist dispatch of the profiled run holds "
                         "(bench.py divides per-dispatch figures by this, not by its own count)")
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    acc = defaultdict(float)
    disp = defaultdict(set)
    for row in csv.DictReader(open(a.csv)):
        k = short(row["Kernel_Name"])
        acc[(k, row["Counter_Name"])] += float(row["Counter_Value"])
        disp[k].add(row["Dispatch_Id"])
    out = {"workload": a.workload, "command": a.command, "kernels": {}}
    if a.note:
        out["note"] = a.note
    for k, ids in disp.items():
        n = len(ids)
        out["kernels"][k] = {c: v / n for (kk, c), v in acc.items() if kk == k}
        out["kernels"][k]["dispatches"] = n
        if a.persist_blocks and "persist" in k:
            out["kernels"][k]["blocks_per_dispatch"] = a.persist_blocks
    json.dump(out, open(a.o, "w"), indent=1)
    for k, v in sorted(out["kernels"].items(), key=lambda kv: -kv[1].get("SQ_INSTS_VALU", 0))[:8]:
        print(f"{k:44s} n={v['dispatches']:4d} " +
              " ".join(f"{c}={x:.4g}" for c, x in v.items() if c not in ("dispatches", "blocks_per_dispatch")))


if __name__ == "__main__":
    main()
