"""VGPR / SGPR / LDS / scratch / code size of every kernel in a built object or
library (the gfx950 code object inside its .hip_fatbin), for occupancy checks
without a GPU.  Usage: python tools/kernel_resources.py FILE [name-regex]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def code_objects(path, tmp):
    """Device code objects in FILE: a .so holds one offload bundle per
    translation unit, concatenated in .hip_fatbin."""
    fb = os.path.join(tmp, "fatbin")
    subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", path, fb],
                   check=True)
    data = open(fb, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    out = []
    for i, st in enumerate(starts):
        part = os.path.join(tmp, f"b{i}")
        with open(part, "wb") as f:
            f.write(data[st: starts[i + 1] if i + 1 < len(starts) else len(data)])
        dev = os.path.join(tmp, f"dev{i}.o")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={dev}"],
                           capture_output=True)
        if r.returncode == 0 and os.path.getsize(dev) > 0:
            out.append(dev)
    return out


def main():
    path = sys.argv[1]
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    notes = syms = ""
    with tempfile.TemporaryDirectory() as tmp:
        for dev in code_objects(path, tmp):
            notes += subprocess.run([f"{LLVM}/llvm-readelf", "--notes", dev], capture_output=True,
                                    text=True).stdout
            syms += subprocess.run([f"{LLVM}/llvm-readelf", "-s", "--wide", dev], capture_output=True,
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
