"""Per-dispatch cycles and effective clock of the SHA-1 kernel from a
rocprofv3 --pmc GRBM_GUI_ACTIVE pass (MI355X_MICROARCH.md 'DVFS give-back':
GRBM_GUI_ACTIVE summed over 8 XCDs)."""
import csv
import statistics
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "sha1" in r["Kernel_Name"] and r["Counter_Name"] == "GRBM_GUI_ACTIVE"]
cyc, clk = [], []
for r in rows:
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    c = float(r["Counter_Value"]) / 8
    cyc.append(c)
    clk.append(c / dur / 1e9)
print(f"{len(rows)} dispatches: cycles median {statistics.median(cyc):.4g}, clock median {statistics.median(clk):.3f} GHz "
      f"(last 10: {statistics.median(clk[-10:]):.3f} GHz, cycles {statistics.median(cyc[-10:]):.4g})")
