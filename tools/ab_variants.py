"""A/B the variant libraries built by tools/build_variants.sh on the bench
workload: one fresh tb_one.py process per (variant, round), rounds
interleaved, best of the rounds.  Usage: ab_variants.py name [name ...]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
names = sys.argv[1:]
best = {}
for rnd in range(int(os.environ.get("AB_ROUNDS", "3"))):
    for nm in names:
        lib = os.path.join(ROOT, "cfd-demo_amd", "lib", "variants", nm, "libcfd_amd.so")
        env = dict(os.environ, CFD_LIB=lib)
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "tb_one.py"), "4096", "5"],
                             env=env, capture_output=True, text=True, timeout=120)
        if out.returncode != 0:
            print(json.dumps({"variant": nm, "error": out.stderr[-400:]}), flush=True)
            sys.exit(1)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        print(json.dumps({"variant": nm, "round": rnd, "us_per_sweep": round(d["us_per_sweep"], 3),
                          "ms_per_step": round(d["ms_per_step"], 4),
                          "state_crc32": d.get("state_crc32")}), flush=True)
        if nm not in best or d["us_per_sweep"] < best[nm]:
            best[nm] = d["us_per_sweep"]
print(json.dumps({"best_us_per_sweep": best}), flush=True)
