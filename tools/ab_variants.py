"""A/B the variant libraries built by tools/build_variants.sh on the bench
workload: one fresh tb_one.py process per (variant, round), rounds
interleaved, best of the rounds.  AB_CMD="parity_one.py 4096 3" times the
reference's control flow instead.  Usage: ab_variants.py name [name ...]"""
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
        cmd = os.environ.get("AB_CMD", "tb_one.py 4096 5").split()
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", cmd[0])] + cmd[1:],
                             env=env, capture_output=True, text=True, timeout=180)
        if out.returncode != 0:
            print(json.dumps({"variant": nm, "error": out.stderr[-400:]}), flush=True)
            sys.exit(1)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        key = "us_per_sweep" if "us_per_sweep" in d else "ms_per_step"
        print(json.dumps({"variant": nm, "round": rnd, "us_per_sweep": d.get("us_per_sweep"),
                          "ms_per_step": round(d["ms_per_step"], 4),
                          "state_crc32": d.get("state_crc32")}), flush=True)
        if nm not in best or d[key] < best[nm]:
            best[nm] = d[key]
print(json.dumps({"best_" + key: best}), flush=True)
