"""CPU: INTEGRATION.md's Rust declarations match the C-ABI.

The drop-in's boundary is include/syncfast_amd.h; INTEGRATION.md shows the
`extern "C"` block a syncfast maintainer adds.  Every entry point the header
declares must appear there as a Rust `fn` with the same number of arguments,
and nothing else may (a stale or misspelt binding would fail to link or,
worse, link with the wrong arity)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _c_arity():
    h = open(os.path.join(ROOT, "include", "syncfast_amd.h")).read()
    out = {}
    for m in re.finditer(r"\n(?:int|const char\s*\*|void|uint64_t)\s*\**\s*(sf_\w+)\s*\(([^;]*?)\);", h, re.S):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("void", "") else args.count(",") + 1
    return out


def _rust_arity():
    t = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    out = {}
    for m in re.finditer(r"\bfn\s+(sf_\w+)\s*\(([^)]*)\)", t, re.S):
        args = [a for a in m.group(2).split(",") if a.strip()]
        out.setdefault(m.group(1), set()).add(len(args))
    return out


def test_every_entry_point_is_declared_for_rust_with_its_arity():
    c, rust = _c_arity(), _rust_arity()
    assert len(c) >= 40
    assert sorted(set(c) - set(rust)) == []
    assert sorted(set(rust) - set(c)) == []
    assert {k: v for k, v in rust.items() if v != {c[k]}} == {}
