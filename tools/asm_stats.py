#!/usr/bin/env python3
"""Static instruction mix of one kernel in a gfx950 assembly file (hipcc --save-temps), per
basic block and in total: VALU (v_*), SALU (s_* but branches / waits), LDS (ds_*), VMEM
(global_* / buffer_*), SMEM (s_load / s_buffer_load), branches, waitcnts.

    python tools/asm_stats.py device-hip-amdgcn-amd-amdhsa-gfx950.s 'k_classifyILi2ELb1ELb1ELi3ELb1ELi512E' [--blocks]
"""
import re
import sys


def kernel_lines(path, pat):
    lines = open(path).read().splitlines()
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^_Z\S*%s\S*:" % re.escape(pat), l):
            start = i
        elif start is not None and l.startswith(".Lfunc_end"):
            return lines[start:i]
    raise SystemExit("kernel not found: " + pat)


def kind(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc")):
        return "branch"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return None


def main():
    path, pat = sys.argv[1], sys.argv[2]
    blocks, cur, name = [], {}, "entry"
    for l in kernel_lines(path, pat):
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            blocks.append((name, cur))
            name, cur = m.group(1), {}
            continue
        t = l.strip().split()
        if not t or t[0].startswith((";", ".")):
            continue
        k = kind(t[0])
        if k:
            cur[k] = cur.get(k, 0) + 1
    blocks.append((name, cur))
    tot = {}
    for n, c in blocks:
        for k, v in c.items():
            tot[k] = tot.get(k, 0) + v
        if "--blocks" in sys.argv and sum(c.values()):
            print("%-16s %s" % (n, " ".join("%s=%d" % kv for kv in sorted(c.items()))))
    print("total", " ".join("%s=%d" % kv for kv in sorted(tot.items())), "blocks=%d" % len(blocks))


if __name__ == "__main__":
    main()
