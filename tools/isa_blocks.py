"""Static instruction mix per basic block of one kernel (gfx950 ISA).

Compiles dcr_kernels.hip to assembly (hipcc -S --cuda-device-only) and prints
every basic block of the named kernel with its VALU / SALU / LDS / VMEM counts
and branch targets, so the per-record instruction budget of a path can be
summed by hand.  DESIGN.md §3 ("What bounds it now") used it on the C2 path
(k_consensus_fast<false,false>, a copy restricted to NT = 3 FULL records).

    python3 tools/isa_blocks.py [kernel-mangled-name] [source.hip]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "_ZN3dcr16k_consensus_fastILb0ELb0EEEvNS_8FastArgsE"
    src = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "duplexumiconsensusreads_amd", "csrc",
                                                             "dcr_kernels.hip")
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        "-S", "--cuda-device-only", "-o", out, src], check=True, stderr=subprocess.DEVNULL)
        s = open(out).read()
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    blocks, cur = [], None
    for line in s[i:j].split("\n"):
        t = line.split(";")[0].strip()
        if not t:
            continue
        if t.endswith(":"):
            cur = {"name": t[:-1], "n": dict.fromkeys("VSLMO", 0), "term": ""}
            blocks.append(cur)
            continue
        if t.startswith("."):
            continue
        if cur is None:
            cur = {"name": "entry", "n": dict.fromkeys("VSLMO", 0), "term": ""}
            blocks.append(cur)
        op = t.split()[0]
        k = ("V" if op.startswith("v_") else "S" if op.startswith("s_") else "L" if op.startswith("ds_")
             else "M" if op.startswith(("buffer", "global", "scratch", "flat")) else "O")
        cur["n"][k] += 1
        if op.startswith(("s_cbranch", "s_branch")):
            cur["term"] += " " + op.replace("s_cbranch_", "") + " " + re.sub(r"\.LBB\d+_", "B", t.split()[1])
    for b in blocks:
        n = b["n"]
        tot = sum(n.values())
        if tot:
            print(f"{re.sub(r'.LBB[0-9]+_', 'B', b['name']):8s} {tot:5d} V{n['V']:4d} S{n['S']:4d} L{n['L']:3d} "
                  f"M{n['M']:3d} |{b['term'][:64]}")


if __name__ == "__main__":
    main()
