#!/usr/bin/env python3
"""Instruction mix of a kernel's hottest loop in a hipcc -S listing.

Finds the function, then every backward branch (s_cbranch_* / s_branch to an
earlier .LBB label inside it); for the largest such loop prints counts by
opcode class.  usage: tools/loop_mix.py <file.s> <kernel-substring> [--all]"""
import collections
import re
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, ln in enumerate(lines) if ln.startswith(key) and
                 ln.split(";")[0].rstrip().endswith(":"))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith("\t.section")
               or re.match(r"^\s*s_endpgm", lines[i]))
    body = lines[start:end + 1]
    labels = {}
    for i, ln in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", ln)
        if m:
            labels[m.group(1)] = i
    loops = []
    for i, ln in enumerate(body):
        m = re.match(r"^\s*s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", ln)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((i - labels[m.group(1)], labels[m.group(1)], i))
    loops.sort(reverse=True)
    show = loops if "--all" in sys.argv else loops[:1]
    for size, a, b in show:
        cnt = collections.Counter()
        for ln in body[a:b + 1]:
            m = re.match(r"^\s+([a-z_0-9]+)", ln)
            if m and not ln.strip().startswith(";") and not m.group(1).startswith("."):
                cnt[m.group(1)] += 1
        valu = sum(v for k, v in cnt.items() if k.startswith("v_"))
        print(f"loop lines {a}-{b}: {sum(cnt.values())} instructions, {valu} VALU")
        for k, v in cnt.most_common():
            print(f"  {v:4d} {k}")


if __name__ == "__main__":
    main()
