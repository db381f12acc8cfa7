"""Per-step time budget from a rocprofv3 kernel trace: kernel time by kernel
and the idle gaps between consecutive dispatches of one queue, over the last
N steps (a step starts at each k_predict_march dispatch).
Usage: python tools/trace_gaps.py TRACE.csv [N]"""
import collections
import csv
import re
import sys


def short(name):
    return re.sub(r"\(.*", "", name.replace("cfd::(anonymous namespace)::", "").replace("void ", ""))


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_predict_march" in r["Kernel_Name"]]
    # steps with no host work inside them (no copy / fill between two
    # predictor dispatches): the last n of those
    clean = [(a, b) for a, b in zip(starts, starts[1:])
             if not any("rocclr" in rows[k]["Kernel_Name"] for k in range(a, b))]
    clean = clean[-n:]
    n = len(clean)
    sel = [rows[k] for a, b in clean for k in range(a, b)]
    tot = collections.Counter()
    cnt = collections.Counter()
    gaps = collections.Counter()
    prev = None
    firsts = {a for a, _ in clean}
    span = sum(int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"]) for a, b in clean)
    for r in sel:
        if prev is not None and "k_predict_march" in r["Kernel_Name"]:
            prev = None   # steps are not contiguous
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        k = short(r["Kernel_Name"])
        tot[k] += e - s
        cnt[k] += 1
        if prev is not None:
            gaps[(short(prev["Kernel_Name"]), k)] += max(0, s - int(prev["End_Timestamp"]))
        prev = r
    print(f"{n} steps, span {span / n / 1e3:.1f} us per step")
    for k, v in tot.most_common():
        print(f"  {v / n / 1e3:8.1f} us/step  {cnt[k] / n:5.1f} calls  {v / cnt[k] / 1e3:7.2f} us/call  {k}")
    g = sum(gaps.values())
    print(f"  {g / n / 1e3:8.1f} us/step  idle between dispatches")
    for (a, b), v in gaps.most_common(6):
        print(f"      {v / n / 1e3:7.1f}  {a} -> {b}")


if __name__ == "__main__":
    main()
