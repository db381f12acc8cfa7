"""VGPR / SGPR / LDS / scratch / code size of every kernel in a built object or
library (the gfx950 code object inside its .hip_fatbin), for occupancy checks
without a GPU.  Usage: python tools/kernel_resources.py FILE [name-regex]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def code_object(path, tmp):
    fb = os.path.join(tmp, "fatbin")
    subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", path, fb],
                   check=True)
    dev = os.path.join(tmp, "dev.o")
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={dev}"], check=True)
    return dev


def main():
    path = sys.argv[1]
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    with tempfile.TemporaryDirectory() as tmp:
        dev = code_object(path, tmp)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", dev], capture_output=True,
                               text=True).stdout
        syms = subprocess.run([f"{LLVM}/llvm-readelf", "-s", "--wide", dev], capture_output=True,
                              text=True).stdout
    size = {}
    for line in syms.splitlines():
        f = line.split()
        if len(f) >= 8 and f[3] == "FUNC":
            size[f[7]] = int(f[2])
    demangle = subprocess.run(["c++filt"], input="\n".join(size), capture_output=True,
                              text=True).stdout.splitlines()
    dm = dict(zip(size, demangle))
    for blk in notes.split("- .agpr_count")[1:]:
        get = lambda k: (re.search(rf"\.{k}:\s+(\S+)", blk) or [None, "?"])[1]
        name = get("name")
        pretty = dm.get(name, name)
        if not pat.search(pretty):
            continue
        short = re.sub(r"\(.*", "", pretty.replace("(anonymous namespace)", "anon"))
        vg = get("vgpr_count")
        waves = 512 // (((int(vg) + 7) // 8) * 8) if vg.isdigit() and int(vg) else "?"
        print(f"vgpr {vg:>4} (<= {waves} waves/SIMD) sgpr {get('sgpr_count'):>4} "
              f"lds {get('group_segment_fixed_size'):>6} scratch {get('private_segment_fixed_size'):>4} "
              f"code {size.get(name, 0):>7}  {short}")


if __name__ == "__main__":
    main()
