"""Instruction mix of a kernel's basic blocks in hipcc -S output.

usage: python tools/isa_loop.py file.s <mangled-name-substring> [--top N]
Prints, per basic block (label), the instruction count and mnemonic histogram
of the N largest blocks (the unrolled inner loops).
"""
import collections
import re
import sys


def blocks(path, name):
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if l.startswith("_Z") and name in l and l.rstrip().endswith(":") is False and ":" in l:
            start = i
            break
        if l.startswith("_Z") and name in l and l.split(";")[0].strip().endswith(":"):
            start = i
            break
    if start is None:
        raise SystemExit("kernel not found")
    cur, out = "entry", collections.OrderedDict()
    out[cur] = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        if l.startswith("; %bb."):          # a fall-through block (no .LBB label)
            cur = l[2:].split(":")[0]
            out[cur] = []
            continue
        s = l.split(";")[0].strip()
        if not s:
            continue
        if s.endswith(":"):
            cur = s[:-1]
            out[cur] = []
            continue
        if s.startswith("."):
            continue
        out[cur].append(s.split()[0])
    return out


def main():
    path, name = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 3
    bl = blocks(path, name)
    for lab, ins in sorted(bl.items(), key=lambda kv: -len(kv[1]))[:top]:
        c = collections.Counter(ins)
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        print(f"== {lab}: {len(ins)} instructions, {valu} VALU")
        for k, v in c.most_common(40):
            print(f"   {v:5d} {k}")


if __name__ == "__main__":
    main()
