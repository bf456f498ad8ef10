"""Where a kernel's scratch spills sit relative to its loops.

usage: python scripts/isa_spill_loops.py listing.s kernel-substring
Prints every loop (back edge) of the kernel with its size in lines and, for
each scratch load/store, the smallest loop that contains it: a spill in a
multi-thousand-line outer loop runs once per group, one in a ~1300-line loop
once per step of a hash path."""
import re
import sys


def main():
    L = open(sys.argv[1]).read().split("\n")
    st = [i for i, l in enumerate(L) if l.startswith("_Z") and sys.argv[2] in l.split(":")[0]][0]
    en = [i for i, l in enumerate(L[st:]) if ".Lfunc_end" in l][0] + st
    K = L[st:en]
    labels = {m.group(1): i for i, l in enumerate(K) for m in [re.match(r"^(\.LBB\d+_\d+):", l)] if m}
    loops = []
    for i, l in enumerate(K):
        m = re.search(r"s_(?:c)?branch\w*\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((labels[m.group(1)], i))
    print("loops (start, lines):", sorted((a, b - a) for a, b in loops))
    for i, l in enumerate(K):
        if "scratch_" in l:
            inner = min([b - a for a, b in loops if a <= i <= b], default=0)
            print(f"{i:6d} {l.strip()[:60]:60s} innermost loop {inner} lines")


if __name__ == "__main__":
    main()
