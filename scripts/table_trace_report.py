"""Report of a per-wave (per-group) trace from scripts/table_trace.py.

usage: python scripts/table_trace_report.py trace.npz [list]
Per SIMD (XCC, SE, CU, SIMD from HW_ID / XCC_ID): the union of its waves'
busy intervals, when it ran out of work; the occupancy over time; the waves
that ended last; compressions per microsecond per SIMD while busy."""
import sys

import numpy as np


def load(path, k):
    t = np.load(path)[k].astype(np.uint64)
    t0 = t[:, 0] | (t[:, 1] << np.uint64(32))
    t1 = t[:, 2] | (t[:, 3] << np.uint64(32))
    ok = t1 > 0
    t, t0, t1 = t[ok], t0[ok], t1[ok]
    base = t0.min()
    s = (t0 - base).astype(np.float64) / 100.0  # s_memrealtime: 100 MHz -> us
    e = (t1 - base).astype(np.float64) / 100.0
    hw, xcc = t[:, 4], t[:, 5]
    simd = (hw >> np.uint64(4)) & np.uint64(3)
    cu = (hw >> np.uint64(8)) & np.uint64(15)
    se = (hw >> np.uint64(13)) & np.uint64(7)
    key = (xcc * np.uint64(1000) + se * np.uint64(100) + cu * np.uint64(4) + simd).astype(np.int64)
    return s, e, key, t[:, 6].astype(np.int64), (t[:, 7] >> np.uint64(8)).astype(np.int64)


def report(path, k):
    s, e, key, nch, nvalid = load(path, k)
    span = e.max()
    print(f"== {path} [{k}]: {len(s)} groups, span {span:.1f} us")
    busy, last = [], []
    for kk in np.unique(key):
        m = key == kk
        o = np.argsort(s[m])
        ss, ee = s[m][o], e[m][o]
        tot, cs, ce = 0.0, ss[0], ee[0]
        for a, b in zip(ss[1:], ee[1:]):
            if a > ce:
                tot += ce - cs
                cs, ce = a, b
            else:
                ce = max(ce, b)
        busy.append(tot + ce - cs)
        last.append(ee.max())
    busy, last = np.array(busy), np.array(last)
    print(f"  SIMDs {len(busy)}: busy/span mean {busy.mean() / span:.4f} min {busy.min() / span:.4f}; "
          f"last end min {last.min():.1f} median {np.median(last):.1f} max {last.max():.1f} us")
    wc = (nch * 1.0).sum()  # wave-compressions (longest lane per group)
    print(f"  wave-compressions {wc:.0f}: {wc / len(busy) / busy.mean():.3f} per SIMD-us while busy")
    T = np.arange(0, span, max(1.0, span / 400))
    occ = np.searchsorted(np.sort(s), T, side="right") - np.searchsorted(np.sort(e), T, side="right")
    print("  resident groups over time:", " ".join(f"{int(T[i])}:{occ[i]}" for i in range(0, len(T), len(T) // 10)))
    late = np.argsort(-e)[:6]
    print("  last to end (group, start, end, compressions):",
          "; ".join(f"{i} {s[i]:.0f}-{e[i]:.0f} {nch[i]}" for i in late))
    d = e - s
    per = d / np.maximum(nch, 1)
    print(f"  us per wave-compression: median {np.median(per):.3f}, p90 {np.percentile(per, 90):.3f}, "
          f"max {per.max():.3f}")


if __name__ == "__main__":
    for k in (sys.argv[2:] or ["cdc", "list4k"]):
        report(sys.argv[1], k)
