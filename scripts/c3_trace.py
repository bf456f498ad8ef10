"""Split a bench.py run's timed region into kernel durations and gaps, from
a rocprofv3 --kernel-trace CSV (scripts/c3_trace.sh).

usage: python scripts/c3_trace.py <kernel_trace.csv> [n_steps]
The timed region is taken as the last n_steps (default 20) launches of the
block kernel (sha1_fixed_kernel or sha1_fixed_chained_kernel) plus every
launch after them (a batch stream's finish)."""
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    big = [i for i, r in enumerate(rows) if "sha1_fixed" in r["Kernel_Name"] and int(r["Grid_Size_X"] if "Grid_Size_X" in r else r.get("Grid_Size", "0")) > 100000]
    first = big[-steps]
    sel = rows[first:]
    t0 = int(sel[0]["Start_Timestamp"])
    t1 = int(sel[-1]["End_Timestamp"])
    busy = 0
    gaps = []
    durs = {}
    prev_end = None
    for r in sel:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0][:60]
        durs.setdefault(name, []).append((e - s) / 1e6)
        if prev_end is not None:
            gaps.append((s - prev_end) / 1e6)
        prev_end = e
        busy += e - s
    print(f"launches {len(sel)}  span {(t1 - t0) / 1e6:.4f} ms  per step {(t1 - t0) / 1e6 / steps:.4f} ms")
    print(f"kernel busy {busy / 1e6:.4f} ms  gaps total {sum(gaps):.4f} ms  max gap {max(gaps) if gaps else 0:.4f}")
    for name, d in durs.items():
        print(f"  {name}: n={len(d)} median {statistics.median(d):.4f} ms  sum {sum(d):.4f}  "
              f"first {d[0]:.4f} last {d[-1]:.4f}")
    print("  last launches:", [f"{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6:.3f}" for r in sel[-4:]])


if __name__ == "__main__":
    main()
