#!/usr/bin/env python3
"""Instruction mix of one kernel's hottest loop from `make asm` output.

  python tools/isa_count.py <file.s> <mangled-name-substring> [--all]

Splits the kernel into basic blocks (labels), finds the loops (a branch back
to an earlier label) and prints, for the loop whose body spans the most
instructions (or every block with --all), the count of VALU / quarter-rate
VALU (32-bit integer multiplies, 64-bit multiply-adds, transcendentals) /
SALU / LDS / VMEM / branch instructions, plus the opcode histogram.  Static
counts: a loop body with rare-path blocks inside counts them once each, so
read the per-block table for what the common path executes."""
import collections
import re
import sys

QUARTER = ("v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32", "v_mad_i64_i32", "v_mul_hi_i32", "v_mul_lo_i32",
           "v_rcp_", "v_sqrt_", "v_rsq_", "v_exp_", "v_log_", "v_sin_", "v_cos_", "v_lshlrev_b64",
           "v_lshrrev_b64", "v_ashrrev_i64")


def load(path, name):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(rf"^\S*{re.escape(name)}\S*:", l))
    body = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end") or l.strip().startswith("s_endpgm"):
            body.append(l)
            break
        body.append(l)
    return body


def blocks(body):
    out, cur, name = [], [], "entry"
    for l in body:
        m = re.match(r"^(\.?[\w$.]+):", l)
        if m:
            out.append((name, cur))
            name, cur = m.group(1), []
            continue
        t = l.strip()
        if not t or t.startswith((";", ".", "//")):
            continue
        cur.append(t.split(";")[0].strip())
    out.append((name, cur))
    return out


def classify(ins):
    op = ins.split()[0]
    if op.startswith("v_"):
        return "valu_q" if op.startswith(QUARTER) else "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    bl = blocks(load(path, name))
    idx = {n: i for i, (n, _) in enumerate(bl)}
    loops = []
    for i, (n, ins) in enumerate(bl):
        for x in ins:
            m = re.match(r"s_c?branch\w*\s+(\.\w+)", x)
            if m and m.group(1) in idx and idx[m.group(1)] <= i:
                loops.append((idx[m.group(1)], i))
    if not loops:
        print("no loop found")
        return
    lo, hi = max(loops, key=lambda t: sum(len(bl[k][1]) for k in range(t[0], t[1] + 1)))
    rng = range(len(bl)) if "--all" in sys.argv else range(lo, hi + 1)
    tot = collections.Counter()
    ops = collections.Counter()
    print(f"loop: blocks {bl[lo][0]} .. {bl[hi][0]}")
    for k in rng:
        n, ins = bl[k]
        c = collections.Counter(classify(x) for x in ins)
        tot.update(c)
        ops.update(x.split()[0] for x in ins)
        print(f"  {n:28s} n={len(ins):4d} " + " ".join(f"{a}={c[a]}" for a in
                                                       ("valu", "valu_q", "salu", "lds", "vmem", "branch", "wait")))
    print("total", dict(tot))
    print("top opcodes:", ", ".join(f"{o}:{c}" for o, c in ops.most_common(40)))


if __name__ == "__main__":
    main()
