"""Sweep Jacobi launch geometries on the GPU, one fresh process per config
(tools/tb_one.py on the bench workload), two passes, best of the two.
TUNE_CONFIGS="kind,T,R[,xcd];..." overrides the list.  Usage: tune_tb.py [n]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
n = sys.argv[1] if len(sys.argv) > 1 else "4096"
configs = [(1, 4, 24), (3, 6, 24), (3, 8, 24)]
if os.environ.get("TUNE_CONFIGS"):
    configs = [tuple(int(x) for x in c.split(",")) for c in os.environ["TUNE_CONFIGS"].split(";")]
configs = [c if len(c) == 4 else tuple(c) + (1,) for c in configs]
best = {}
for rnd in range(2):
    for kind, t, r, x in configs:
        env = dict(os.environ, CFD_TB_KIND=str(kind), CFD_TEMPORAL=str(t), CFD_XCD_REMAP=str(x))
        env.pop("CFD_TB_BPC", None)
        env.pop("CFD_TB_ROWS", None)
        if r > 0:
            env["CFD_TB_ROWS"] = str(r)
        else:
            env["CFD_TB_BPC"] = str(-r)
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "tb_one.py"), n, "5"],
                             env=env, capture_output=True, text=True, timeout=120)
        if out.returncode != 0:
            print(json.dumps({"config": [kind, t, r, x], "error": out.stderr[-400:]}), flush=True)
            continue
        d = json.loads(out.stdout.strip().splitlines()[-1])
        k = (kind, t, r, x)
        if k not in best or d["ms_per_step"] < best[k]["ms_per_step"]:
            best[k] = d
for (kind, t, r, x), d in best.items():
    print(json.dumps({"kind": kind, "T": t, "R": r, "xcd": x, "us_per_sweep": round(d["us_per_sweep"], 3),
                      "ms_per_step": round(d["ms_per_step"], 4), "kernel": d["kernel"]}), flush=True)
