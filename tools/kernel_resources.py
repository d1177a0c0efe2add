"""Per-kernel register / scratch / LDS usage of one csrc/*.hip file, from hipcc's own code-object
metadata (no GPU): the device assembly (-S --offload-device-only) is parsed for the AMDHSA
metadata block of every kernel.

    python tools/kernel_resources.py news_x2.hip [-DFLAG ...]     # table on stdout
    python tools/kernel_resources.py news_x2.hip --asm out.s       # also keep the assembly

The file's own FILE_FLAGS (miner_amd/build.py) are applied, so the numbers are the product build's.
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def device_asm(name, extra=(), out=None):
    from miner_amd.build import FILE_FLAGS, hipcc
    src = os.path.join(ROOT, "miner_amd", "csrc", name)
    out = out or f"/tmp/{name}.s"
    cmd = [hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-Wno-pass-failed", *FILE_FLAGS.get(name, []),
           *extra, "-I", os.path.join(ROOT, "include"), "--offload-device-only", "-S", src, "-o", out]
    subprocess.run(cmd, check=True, capture_output=True)
    return out


def parse(path):
    text = open(path).read()
    meta = text[text.rfind("amdhsa.kernels:"):]
    rows = []
    for blk in re.split(r"\n  - ", meta)[1:]:
        f = dict(re.findall(r"^\s*\.(\w+):\s+(\S+)", blk, re.M))
        rows.append({"name": f.get("name", "?"), "vgpr": int(f.get("vgpr_count", 0)),
                     "agpr": int(f.get("agpr_count", 0)), "sgpr": int(f.get("sgpr_count", 0)),
                     "vgpr_spill": int(f.get("vgpr_spill_count", 0)), "sgpr_spill": int(f.get("sgpr_spill_count", 0)),
                     "scratch": int(f.get("private_segment_fixed_size", 0)),
                     "lds_static": int(f.get("group_segment_fixed_size", 0))})
    return rows


def demangle(names):
    try:
        r = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-cxxfilt"], input="\n".join(names), capture_output=True,
                           text=True, check=True)
        return r.stdout.splitlines()
    except (OSError, subprocess.SubprocessError):
        return names


if __name__ == "__main__":
    args = sys.argv[1:]
    asm = None
    if "--asm" in args:
        i = args.index("--asm")
        asm = args[i + 1]
        args = args[:i] + args[i + 2:]
    name, extra = args[0], args[1:]
    rows = parse(device_asm(name, extra, asm))
    for r, dn in zip(rows, demangle([r["name"] for r in rows])):
        dn = re.sub(r"\(anonymous namespace\)::", "", dn).replace("(X2Params)", "")
        print(f"{r['vgpr']:4d} vgpr {r['agpr']:4d} agpr {r['sgpr']:4d} sgpr  spill v{r['vgpr_spill']:<3d} "
              f"s{r['sgpr_spill']:<3d} scratch {r['scratch']:4d} B  {dn}")
