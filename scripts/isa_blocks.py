"""Instruction histogram of the largest basic blocks of one kernel in a hipcc --save-temps
.s file (design aid for the Viterbi body).  usage: isa_blocks.py file.s kernel_symbol [n]"""
import collections
import re
import sys


def main(path, sym, nblocks=6):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur, name = [], [], "entry"
    for l in lines[start + 1:end]:
        t = l.strip()
        if re.match(r"^(\.LBB\S+:|; %bb\.\d+:)", t):
            blocks.append((name, cur))
            name, cur = t.split()[0] if t.startswith(".LBB") else t.split(":")[0], []
            continue
        if not t or t.startswith(";") or t.startswith("."):
            continue
        cur.append(t.split()[0])
    blocks.append((name, cur))
    blocks.sort(key=lambda b: -len(b[1]))
    for name, ins in blocks[:int(nblocks)]:
        c = collections.Counter(ins)
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        print(f"{name}: {len(ins)} instructions, {valu} VALU, {c['ds_swizzle_b32']} swizzle, "
              f"{sum(v for k, v in c.items() if k.startswith('ds_write'))} ds_write, {c['v_pk_min_u16']} pk_min")
        print("   ", ", ".join(f"{k} {v}" for k, v in c.most_common(14)))


if __name__ == "__main__":
    main(*sys.argv[1:])
