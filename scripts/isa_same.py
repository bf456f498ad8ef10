"""Compare kernels' machine code between two `make isa` listings (.s).

usage: python scripts/isa_same.py OLD.s NEW.s [kernel-substring ...]
Prints, per kernel whose symbol contains a substring (default: the fixed-
tiling, chained and staged kernels), whether its instruction text is
identical.  Used to keep sha1_fixed_kernel's code unchanged while other
kernels of the same translation unit change."""
import re
import sys


def bodies(path):
    out, cur, name = {}, None, None
    for line in open(path):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            name, cur = m.group(1), []
            continue
        if name and line.startswith(".Lfunc_end"):
            out[name] = [l for l in cur if not l.lstrip().startswith(";")]
            name = None
            continue
        if name is not None:
            # basic-block labels carry the function's index in the TU
            # (.LBB<fn>_<bb>): another kernel added before it renumbers them
            cur.append(re.sub(r"\.LBB\d+_", ".LBB_", line.split(";")[0].rstrip()))
    return out


def main():
    a, b = bodies(sys.argv[1]), bodies(sys.argv[2])
    subs = sys.argv[3:] or ["sha1_fixed_kernel", "sha1_fixed_chained_kernel", "sha1_staged_kernel"]
    ok = True
    for k in sorted(a):
        if any(s in k for s in subs):
            same = k in b and a[k] == b[k]
            ok &= same
            print(f"{'same' if same else 'DIFFERENT'} {len(a[k])} lines {k}")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
