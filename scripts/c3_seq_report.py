"""Report of scripts/c3_seq.py's kernel trace: mean launch duration per
segment and round.  usage: python scripts/c3_seq_report.py <kernel_trace.csv> n_libs [K]"""
import csv
import statistics
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "sha1" in r["Kernel_Name"]]
    nlib = int(sys.argv[2])
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    st = [int(r["Start_Timestamp"]) for r in rows]
    en = [int(r["End_Timestamp"]) for r in rows]
    dur = [(e - s) / 1e6 for s, e in zip(st, en)]
    per_lib = K + (K - 1) + 2 + 1  # blocks_only, pushes, two halves, finish
    per_round = K + nlib * per_lib
    rounds = len(rows) // per_round
    acc = {}
    for rd in range(1, rounds):  # round 0 warms up
        b = rd * per_round
        line = [f"plain {statistics.mean(dur[b:b + K]):.4f}"]
        acc.setdefault("plain", []).append(statistics.mean(dur[b:b + K]))
        for j in range(nlib):
            o = b + K + j * per_lib
            bo = statistics.mean(dur[o:o + K])
            s0 = o + K
            ch = statistics.mean(dur[s0 + 1:s0 + K - 1])  # pushes with chain jobs (not the first)
            span = (en[s0 + per_lib - K - 1] - st[s0]) / 1e6 / K
            line.append(f"lib{j}: blocks_only {bo:.4f} chained {ch:.4f} halves {dur[s0 + K - 1] + dur[s0 + K]:.4f} "
                        f"finish {dur[s0 + K + 1]:.4f} stream/batch {span:.4f}")
            for k, v in (("bo", bo), ("ch", ch), ("span", span)):
                acc.setdefault(f"lib{j}:{k}", []).append(v)
        print(f"round {rd}: " + " | ".join(line))
    print("means over rounds 1..: " + "  ".join(f"{k} {statistics.mean(v):.4f}" for k, v in acc.items()))


if __name__ == "__main__":
    main()
