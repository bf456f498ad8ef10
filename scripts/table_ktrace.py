"""Per-launch kernel times of an interleaved scripts/cdc_ab.py run under
rocprofv3 --kernel-trace (no counters): the dispatch order is cdc_ab.py's
(for each round, for each list, for each library, CDC_REPS calls), so every
sha1_table_kernel launch is attributed to its library and list, with the
sort kernels before it and the gaps around it.
usage: python scripts/table_ktrace.py kernel_trace.csv LISTS NLIBS REPS ROUNDS [rot]
(rot: cdc_ab.py rotated the library order every round, its default since s22).
A library whose sort ends with group_geo_kernel (round 5) counts it in the
sort's time."""
import csv
import statistics
import sys


def main():
    path, lists, nlibs, reps, rounds = sys.argv[1], sys.argv[2].split(","), int(sys.argv[3]), int(sys.argv[4]), \
        int(sys.argv[5])
    rot = len(sys.argv) > 6 and sys.argv[6] == "rot"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    calls, cur, fixed = [], [], []
    for r in rows:
        n = r["Kernel_Name"]
        if "sha1_fixed_kernel" in n:
            fixed.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        if "class_hist_kernel" in n:
            cur = [r]
        elif cur and ("class_scan" in n or "class_scatter" in n or "group_geo" in n):
            cur.append(r)
        elif "sha1_table_kernel<128, false>" in n and len(cur) in (3, 4):
            cur.append(r)
            calls.append(cur)
            cur = []
    # cdc_ab.py makes list calls only in its timed rounds (the clock ramp uses the fixed kernel)
    need = rounds * len(lists) * nlibs * reps
    calls = calls[-need:]
    res = {}
    i = 0
    for _r in range(rounds):
        for k in lists:
            for pos in range(nlibs):
                lib = (pos + _r) % nlibs if rot else pos
                for _ in range(reps):
                    c = calls[i]
                    i += 1
                    t = [(int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in c]
                    res.setdefault((lib, k), []).append(((t[-1][1] - t[-1][0]) / 1e3, (t[-1][0] - t[0][0]) / 1e3,
                                                          (t[-1][1] - t[0][0]) / 1e3))
    if fixed:
        print(f"fixed kernel median {statistics.median(fixed):.1f} us ({len(fixed)} launches)")
    for (lib, k), v in sorted(res.items()):
        print(f"lib{lib} {k}: table kernel median {statistics.median(x[0] for x in v):.1f} us, sort+gaps "
              f"{statistics.median(x[1] for x in v):.1f} us, call {statistics.median(x[2] for x in v):.1f} us "
              f"({len(v)} calls)")


if __name__ == "__main__":
    main()
