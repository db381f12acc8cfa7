"""A/B environment settings of the library on the bench workload: one fresh
tools/tb_one.py process per (setting, round), rounds interleaved, best of
three (AB_ROUNDS), with the median.  AB_CMD="parity_one.py 4096 3" (or AB_N=8192)
changes the workload.
Usage: ab_env.py "NAME=VAL[,NAME=VAL]" ...   ("" = defaults)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
specs = sys.argv[1:]
best, allv = {}, {}
for rnd in range(int(os.environ.get("AB_ROUNDS", "3"))):
    for sp in specs:
        env = dict(os.environ)
        for kv in filter(None, sp.split(",")):
            k, v = kv.split("=", 1)
            env[k] = v
        cmd = os.environ.get("AB_CMD", "tb_one.py " + os.environ.get("AB_N", "4096") + " 5").split()
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", cmd[0])] + cmd[1:],
                             env=env, capture_output=True, text=True, timeout=180)
        if out.returncode != 0:
            print(json.dumps({"setting": sp, "error": out.stderr[-400:]}), flush=True)
            sys.exit(1)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        key = "us_per_sweep" if "us_per_sweep" in d else "ms_per_step"
        print(json.dumps({"setting": sp, "round": rnd, "us_per_sweep": d.get("us_per_sweep"),
                          "ms_per_step": round(d["ms_per_step"], 4),
                          "geometry": d.get("geometry"), "persist_blocks": d.get("persist_blocks"),
                          "steals": d.get("persist_steals"),
                          "crc": d.get("state_crc32")}), flush=True)
        best[sp] = min(best.get(sp, 1e9), d[key])
        allv.setdefault(sp, []).append(d[key])
med = {k: sorted(v)[len(v) // 2] for k, v in allv.items()}
print(json.dumps({"best_" + key: best, "median_" + key: med}), flush=True)
