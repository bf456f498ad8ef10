"""Compare the largest basic block (the LDS main loop) of the chained kernel
with the plain fixed kernel's: opcode sequence and full text (registers).
usage: python scripts/isa_loop_cmp.py file.s"""
import difflib
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
import isa_hist as h  # noqa: E402

PLAIN = "_ZN2sf17sha1_fixed_kernelILi128ELi1ELb0EEEvPKhmjmPhNS_11PadScheduleEPj"


def main():
    s = open(sys.argv[1]).read()
    m = re.search(r"^(_ZN2sf25sha1_fixed_chained_kernelILi128EE\S*):", s, re.M)
    A, B = h.body(s, PLAIN), h.body(s, m.group(1))
    ba, bb = h.blocks(A), h.blocks(B)
    la = max(ba, key=lambda k: len(ba[k]))
    lb = max(bb, key=lambda k: len(bb[k]))
    a, b = ba[la], bb[lb]
    r = difflib.SequenceMatcher(a=a, b=b, autojunk=False).ratio()
    print(f"hot loop: plain {la} {len(a)} ops, chained {lb} {len(b)} ops, same sequence {a == b}, ratio {r:.4f}")


if __name__ == "__main__":
    main()
