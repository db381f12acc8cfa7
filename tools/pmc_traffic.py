"""Per-dispatch HBM-side traffic of each kernel from two rocprofv3 PMC passes
(FETCH_SIZE and WRITE_SIZE, each its own run), corrected as
/opt/skills/guides/MI355X_MICROARCH.md §HBM prescribes for gfx950:
FETCH_SIZE (KiB) reports half the bytes of wide coalesced streaming reads, so
bytes read = 2 x FETCH_SIZE x 1024; WRITE_SIZE (KiB) is exact for 16-B and
8-B-per-lane streaming stores.  Writes a JSON summary that bench.py reads to
fill roofline.traffic.

    python tools/pmc_traffic.py fetch_counter_collection.csv \
        write_counter_collection.csv --workload 4096x4096 -o profiles/r1/pmc_traffic.json
"""
import argparse
import csv
import json
from collections import defaultdict


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").replace("cfd::", "")\
        .split("(")[0]


def per_dispatch(path, counter):
    acc, n = defaultdict(float), defaultdict(set)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter:
            continue
        k = short(row["Kernel_Name"])
        acc[k] += float(row["Counter_Value"])
        n[k].add(row["Dispatch_Id"])
    return {k: acc[k] / len(n[k]) for k in acc}, {k: len(v) for k, v in n.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--command", default="")
    ap.add_argument("-o", "--out", required=True)
    ap.add_argument("--persist-blocks", type=int, default=0,
                    help="T-sweep blocks one k_jacobi_persist dispatch of the profiled run holds "
                         "(bench.py divides per-dispatch bytes by this, not by its own count)")
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    fetch, nf = per_dispatch(a.fetch_csv, "FETCH_SIZE")
    write, nw = per_dispatch(a.write_csv, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        rd = 2.0 * fetch.get(k, 0.0) * 1024.0
        wr = write.get(k, 0.0) * 1024.0
        kernels[k] = {"read_bytes": rd, "write_bytes": wr, "traffic_bytes": rd + wr,
                      "dispatches": max(nf.get(k, 0), nw.get(k, 0))}
        if a.persist_blocks and "persist" in k:
            kernels[k]["blocks_per_dispatch"] = a.persist_blocks
    out = {"workload": a.workload, "command": a.command,
           "correction": "read = 2 x FETCH_SIZE KiB (gfx950 half-count of wide streaming reads), "
                         "write = WRITE_SIZE KiB; per dispatch, averaged",
           "kernels": kernels}
    if a.note:
        out["note"] = a.note
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    for k, v in kernels.items():
        print(f"{k:50s} {v['traffic_bytes'] / 1e6:10.2f} MB/dispatch  n={v['dispatches']}")


if __name__ == "__main__":
    main()
