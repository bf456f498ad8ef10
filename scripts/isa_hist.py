"""Opcode histograms of two kernels in an ISA listing (make isa), and of
their hottest loop bodies.  usage: python scripts/isa_hist.py file.s symA symB"""
import collections
import re
import sys


def body(s, name):
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    return s[i:j]


def ops(t):
    out = []
    for ln in t.split("\n"):
        ln = ln.strip()
        if not ln or ln.startswith((".", ";", "_")) or re.match(r"^\S+:", ln):
            continue
        out.append(ln.split()[0])
    return out


def blocks(t):
    """basic blocks: label -> opcode list"""
    cur, res = "entry", collections.OrderedDict()
    res[cur] = []
    for ln in t.split("\n"):
        m = re.match(r"^(\.LBB\S+):", ln.strip())
        if m:
            cur = m.group(1)
            res[cur] = []
            continue
        res[cur] += ops(ln)
    return res


def main():
    s = open(sys.argv[1]).read()
    A, B = body(s, sys.argv[2]), body(s, sys.argv[3])
    ha, hb = collections.Counter(ops(A)), collections.Counter(ops(B))
    print("total", sum(ha.values()), sum(hb.values()))
    for k in sorted(set(ha) | set(hb), key=lambda k: -(ha[k] + hb[k]))[:30]:
        print(f"  {k:28s} {ha[k]:6d} {hb[k]:6d}")
    for name, t in (("A", A), ("B", B)):
        bl = blocks(t)
        big = sorted(bl.items(), key=lambda kv: -len(kv[1]))[:4]
        print(name, "largest blocks:", [(k, len(v)) for k, v in big])


if __name__ == "__main__":
    main()
