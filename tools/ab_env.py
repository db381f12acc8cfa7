"""A/B environment settings of the library on the bench workload: one fresh
tools/tb_one.py process per (setting, round), rounds interleaved, best of
three.  Usage: ab_env.py "NAME=VAL[,NAME=VAL]" ...   ("" = defaults)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
specs = sys.argv[1:]
best = {}
for rnd in range(3):
    for sp in specs:
        env = dict(os.environ)
        for kv in filter(None, sp.split(",")):
            k, v = kv.split("=", 1)
            env[k] = v
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "tb_one.py"), os.environ.get("AB_N", "4096"), "5"],
                             env=env, capture_output=True, text=True, timeout=120)
        if out.returncode != 0:
            print(json.dumps({"setting": sp, "error": out.stderr[-400:]}), flush=True)
            sys.exit(1)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        print(json.dumps({"setting": sp, "round": rnd, "us_per_sweep": round(d["us_per_sweep"], 3),
                          "ms_per_step": round(d["ms_per_step"], 4)}), flush=True)
        best[sp] = min(best.get(sp, 1e9), d["us_per_sweep"])
print(json.dumps({"best_us_per_sweep": best}), flush=True)
