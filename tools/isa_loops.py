"""Instruction mix of a kernel's loops from its ISA (hipcc --save-temps .s file).

    python tools/isa_loops.py FILE.s KERNEL_SUBSTRING [--min 40]

Splits the kernel's function body into basic blocks (labels), finds backward branches (a
branch to a label defined earlier = a loop from that label to the branch) and prints each
loop's instruction counts by class -- VALU (v_*), SALU (s_* without branches / waits),
VMEM (buffer_* / global_*), LDS (ds_*), DPP-modified VALU, waitcnt -- plus the counts of
the named opcodes that dominate FAST's sweep (lerp, alignbyte, bitop3, bfi, perm).  Used for
DESIGN.md's per-phase instruction budget.
"""
import argparse
import collections
import re


def classify(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--min", type=int, default=40, help="smallest loop (instructions) to print")
    args = ap.parse_args()
    lines = open(args.asm).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(args.kernel + ":"))
    body = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end") or "-- End function" in l:
            break
        body.append(l)
    labels = {}
    insts = []          # (index, opcode, text)
    for l in body:
        s = l.strip()
        if not s or s.startswith(";") or s.startswith("."):
            m = re.match(r"^(\.LBB[\w_]+):", s)
            if m:
                labels[m.group(1)] = len(insts)
            continue
        op = s.split()[0]
        insts.append((op, s))
    loops = []
    for i, (op, s) in enumerate(insts):
        if op.startswith(("s_cbranch", "s_branch")):
            tgt = s.split()[-1]
            if tgt in labels and labels[tgt] <= i:
                loops.append((labels[tgt], i))
    key_ops = ("v_lerp_u8", "v_alignbyte_b32", "v_bitop3_b32", "v_bfi_b32", "v_perm_b32",
               "v_mov_b32_dpp", "v_not_b32", "v_mbcnt_lo_u32_b32", "v_add_u32", "v_cndmask_b32")
    print(f"{args.kernel}: {len(insts)} instructions, {len(loops)} backward branches")
    for a, b in sorted(set(loops), key=lambda t: -(t[1] - t[0])):
        if b - a < args.min:
            continue
        c = collections.Counter(classify(op) for op, _ in insts[a:b + 1])
        dpp = sum(1 for op, s in insts[a:b + 1] if "dpp" in op or " row_" in s or "wave_" in s)
        named = collections.Counter(op for op, _ in insts[a:b + 1] if op in key_ops)
        print(f"loop [{a}, {b}] len {b - a + 1}: " + " ".join(f"{k}={v}" for k, v in sorted(c.items()))
              + f" dpp={dpp} | " + " ".join(f"{k}={v}" for k, v in sorted(named.items())))


if __name__ == "__main__":
    main()
