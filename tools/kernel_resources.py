"""Per-kernel resource usage (VGPR/AGPR counts, spills, LDS, scratch) of an in-tree library's
gfx950 code object, read from the AMDGPU metadata notes (llvm-readelf --notes).
   usage: python tools/kernel_resources.py [lib.so] [name-filter]"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")


def kernels(lib):
    with tempfile.TemporaryDirectory() as d:
        fat, co = Path(d) / "fat.bin", Path(d) / "k.co"
        subprocess.run([LLVM / "llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fat], check=True)
        subprocess.run([LLVM / "clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([LLVM / "llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    # one metadata map per kernel: keys sorted, '.args' first; a kernel's entry starts at '.agpr_count'
    out, cur = [], None
    for line in notes.splitlines():
        m = re.match(r"\s*-?\s*\.(\w+):\s*(.*)$", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "agpr_count":
            cur = {}
            out.append(cur)
        if cur is not None and k in ("agpr_count", "group_segment_fixed_size", "name",
                                     "private_segment_fixed_size", "vgpr_count", "vgpr_spill_count",
                                     "sgpr_count", "sgpr_spill_count", ".symbol"):
            cur.setdefault(k, v)
    return out


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines()


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else str(Path(__file__).resolve().parents[1] /
                                                     "convex-mpc-unitree-go2_amd/cmpc/lib/libcmpc.so")
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    ks = [k for k in kernels(lib) if "name" in k]
    for k, dn in zip(ks, demangle([k["name"] for k in ks])):
        if flt not in dn:
            continue
        short = re.sub(r"\(.*\)$", "", dn).replace("cmpc::", "")
        print(f"{short:46s} vgpr {k.get('vgpr_count'):>4} agpr {k.get('agpr_count'):>4} "
              f"vgpr_spill {k.get('vgpr_spill_count'):>5} lds {k.get('group_segment_fixed_size'):>6} "
              f"scratch {k.get('private_segment_fixed_size'):>5}")


if __name__ == "__main__":
    main()
