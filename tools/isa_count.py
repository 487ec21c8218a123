"""Instruction counts of the hot loops of the shipped harmonic kernels, read from the
gfx950 assembly the library is built from: the staged near
field's column loop (k_near_hs<5, 2, 2, true, ...>: per lane 2 columns x 4 rows = 8
entries per iteration) and the cluster M2L's directed (2 pairs) and canonical (2 pairs,
both products) loops (k_top_m2l_hc<5, 1, 3, 0, ...>: per lane 4 rows of a column = 4
entries per pair).  Counts are wave instructions per lane-entry.
A loop is a back-edge to an earlier label; the hot one is the innermost loop with the
kernel's signature instructions (near: v_rsq_f64 and global loads, no LDS atomics;
M2L: v_rsq_f64, the canonical one with ds_add_f64).
usage: isa_count.py [harmonic.s]  (default: compiles aniso_amd/csrc/harmonic.hip)"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def assembly():
    if len(sys.argv) > 1:
        return open(sys.argv[1]).read()
    out = os.path.join(tempfile.gettempdir(), "aniso_harmonic_isa.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                    "-munsafe-fp-atomics", "--cuda-device-only", "-S", "harmonic.hip", "-o", out],
                   cwd=os.path.join(ROOT, "aniso_amd", "csrc"), check=True, stderr=subprocess.DEVNULL)
    return open(out).read()


def body(asm, prefix):
    lines = asm.split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(prefix) and l.rstrip().endswith(":")
                 or (l.startswith(prefix) and ": ;" in l))
    end = start
    while not lines[end].startswith(".Lfunc_end"):
        end += 1
    return lines[start:end]


def loops(b):
    lab = {l.split(":")[0]: i for i, l in enumerate(b) if re.match(r"^\.LBB\d+_\d+:", l)}
    out = []
    for i, l in enumerate(b):
        m = re.search(r"s_(cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
        if m and m.group(2) in lab and lab[m.group(2)] < i:
            out.append((lab[m.group(2)], i))
    return out


def count(b, a, z):
    c = collections.Counter()
    for l in b[a:z]:
        t = l.strip()
        if t and not t.startswith((";", ".")):
            c[t.split()[0]] += 1
    return c


def summary(c, entries):
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    f64 = sum(v for k, v in c.items() if k.startswith("v_") and "f64" in k)
    vmem = sum(v for k, v in c.items() if k.startswith(("global_load", "buffer_load")))
    lds = sum(v for k, v in c.items() if k.startswith("ds_"))
    return {"entries_per_iteration": entries, "valu": valu, "valu_per_entry": round(valu / entries, 2),
            "fp64_valu_per_entry": round(f64 / entries, 2), "vmem_loads": vmem, "lds_ops": lds,
            "top": dict(c.most_common(8))}


def pick(b, want, avoid=None):
    best = None
    for a, z in loops(b):
        c = count(b, a, z)
        if all(c[k] > 0 for k in want) and not (avoid and c[avoid] > 0):
            if best is None or z - a < best[1] - best[0]:  # the innermost such loop
                best = (a, z)
    return best


def main():
    asm = assembly()
    res = {}
    nb = body(asm, "_ZN5aniso9k_near_hsILi5ELi2ELi2ELb1ELb0ELb0ELb0EEEvNS_10NearHsArgsE")
    a, z = pick(nb, ["v_rsq_f64_e32", "global_load_dwordx4"], "ds_add_f64")
    res["k_near_hs<5,2,2,fused> column loop"] = summary(count(nb, a, z), 8)
    mb = body(asm, "_ZN5aniso12k_top_m2l_hcILi5ELi1ELi3ELi0ELb0ELb0ELb0EEEvNS_6UpArgsENS_7TopArgsENS_6HcArgsENS_10NearHsArgsE")
    a, z = pick(mb, ["v_rsq_f64_e32", "ds_add_f64"])
    res["k_top_m2l_hc<5> canonical loop (2 pairs, both products)"] = summary(count(mb, a, z), 2 * 4)
    a, z = pick(mb, ["v_rsq_f64_e32", "global_load_dwordx4"], "ds_add_f64")
    res["k_top_m2l_hc<5> directed loop (2 pairs)"] = summary(count(mb, a, z), 2 * 4)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
