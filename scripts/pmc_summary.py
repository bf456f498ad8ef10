"""Per-launch means of rocprofv3 --pmc counters for one kernel, plus the
effective clock (GRBM_GUI_ACTIVE / XCDs / duration) when that counter is
present.  Usage: pmc_summary.py KERNEL_SUBSTRING name=csv [name=csv ...]
(the csv is rocprofv3's pmc_counter_collection.csv)."""
import collections
import csv
import sys

XCDS = 8


def summarise(path, kernel):
    agg = collections.defaultdict(list)
    dur = {}
    for r in csv.DictReader(open(path)):
        if kernel not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    out = {k: sum(v) / len(v) for k, v in agg.items()}
    ms = sorted(dur.values())
    out["launches"] = len(ms)
    out["median_ms"] = ms[len(ms) // 2] if ms else float("nan")
    if "GRBM_GUI_ACTIVE" in out and ms:
        out["clock_ghz"] = out["GRBM_GUI_ACTIVE"] / XCDS / (sum(ms) / len(ms)) / 1e6
    return out


def main():
    kernel = sys.argv[1]
    for arg in sys.argv[2:]:
        name, path = arg.split("=", 1)
        s = summarise(path, kernel)
        print(name, " ".join(f"{k}={v:.5g}" for k, v in sorted(s.items())))


if __name__ == "__main__":
    main()
