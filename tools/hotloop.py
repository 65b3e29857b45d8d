"""Static instruction count of a kernel's hot loop from gfx950 assembly.

Usage: python tools/hotloop.py file.s [kernel-substring] [--first] [-v]
Finds the loop (by label) whose straight-line path contains the most
v_bitop3_b32 (the Philox rounds) and prints the instruction mix along the
fall-through path from the loop header to the first branch back or out that
has consumed the Philox block.  Only a rough guide: measure on the GPU.
"""
import collections
import re
import sys


def kernel_lines(asm, want):
    out = {}
    for m in re.finditer(r"^(_Z[^:\s]+):", asm, re.M):
        name = m.group(1)
        if want and want not in name:
            continue
        end = asm.index(".Lfunc_end", m.end())
        out[name] = asm[m.end():end].split("\n")
    return out


def blocks(lines):
    bl, cur, name = [], [], "entry"
    for ln in lines:
        if re.match(r"^\.LBB\S+:", ln):
            bl.append((name, cur))
            name, cur = ln.split(":")[0], []
        elif ln.startswith("\t") and not ln.strip().startswith((".", ";")):
            cur.append(ln.strip())
    bl.append((name, cur))
    return bl


def classify(ins):
    op = ins.split()[0]
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main():
    asm = open(sys.argv[1]).read()
    want = sys.argv[2] if len(sys.argv) > 2 else "k_encode_prune"
    for name, lines in kernel_lines(asm, want).items():
        bl = blocks(lines)
        # the main loop: the first block holding one whole Philox-10 (~20 bitop3)
        cands = [i for i in range(len(bl)) if sum("v_bitop3_b32" in x for x in bl[i][1]) >= 16]
        if not cands:
            continue
        best = cands[0] if "--first" in sys.argv else max(
            cands, key=lambda i: sum("v_bitop3_b32" in x for x in bl[i][1]))
        # follow fall-through until the block ends with an unconditional branch or
        # a conditional branch we treat as rarely taken (execz/vccnz skip targets
        # are not followed: we only count the straight path)
        path, i = [], best
        while i < len(bl):
            path += bl[i][1]
            last = bl[i][1][-1] if bl[i][1] else ""
            if last.startswith("s_branch") or len(path) > 2000:
                break
            i += 1
            if last.startswith("s_cbranch_vccnz") or last.startswith("s_cbranch_scc"):
                break
        c = collections.Counter(classify(x) for x in path)
        ops = collections.Counter(x.split()[0] for x in path)
        print(f"{name[:70]}\n  hot path from {bl[best][0]}: {len(path)} instr  {dict(c)}")
        if "-v" in sys.argv:
            for op, n in ops.most_common():
                print(f"    {op:28s} {n}")


if __name__ == "__main__":
    main()
