"""FETCH_SIZE / WRITE_SIZE calibration from tools/probes/fetch_calib.hip.

Each probe kernel moves a known byte count (printed by the probe) with one
access width; the ratio known bytes / (counter KiB x 1024) is the factor that
turns the counter into bytes for that width on gfx950 (the guide documents
x2 for 16-B-per-lane reads only, MI355X_MICROARCH.md §HBM).

    python tools/pmc_calib.py fetch.csv write.csv --bytes N -o profiles/r3/fetch_calibration.json
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import per_dispatch  # noqa: E402

WIDTH = {"k_rd_buf32": "buffer_load_b32 (4 B/lane)", "k_rd_buf64": "buffer_load_b64 (8 B/lane)",
         "k_rd_buf128": "buffer_load_b128 (16 B/lane)", "k_rd_flat64": "global_load_dwordx2 (8 B/lane)",
         "k_rd_flat128": "global_load_dwordx4 (16 B/lane)",
         "k_wr_buf64": "buffer_store_b64 (8 B/lane)", "k_wr_flat128": "global_store_dwordx4 (16 B/lane)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--bytes", type=float, required=True)
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    fetch, _ = per_dispatch(a.fetch_csv, "FETCH_SIZE")
    write, _ = per_dispatch(a.write_csv, "WRITE_SIZE")
    res = {}
    for k, w in WIDTH.items():
        ent = {"access": w, "known_bytes": a.bytes}
        if k in fetch:
            ent["fetch_size_bytes"] = fetch[k] * 1024.0
            ent["read_factor"] = a.bytes / (fetch[k] * 1024.0) if fetch[k] else None
        if k in write:
            ent["write_size_bytes"] = write[k] * 1024.0
            ent["write_factor"] = a.bytes / (write[k] * 1024.0) if write[k] else None
        res[k] = ent
    out = {"probe": "tools/probes/fetch_calib.hip", "buffer_bytes": a.bytes,
           "note": "factor = known bytes / counter bytes (counter KiB x 1024), per dispatch "
                   "(averaged over a warm-up and a measured dispatch of each kernel)",
           "kernels": res}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    for k, v in res.items():
        print(f"{k:14s} {v['access']:34s} read x{v.get('read_factor') or 0:6.3f}  "
              f"write x{v.get('write_factor') or 0:6.3f}")


if __name__ == "__main__":
    main()
