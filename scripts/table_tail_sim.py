"""Schedule model of the explicit-list kernel's tail.

usage: python scripts/table_tail_sim.py trace.npz [list]

Takes the group lengths (compressions) of a traced launch in the sort's order
and replays the hardware's dispatch under a simple model: 1024 SIMDs x 3
slots; the first 3072 waves land on SIMD w % 1024 (what the traces show);
a SIMD runs its waves oldest first, one at a time (the sequencer's age
arbitration); a slot freed when a wave ends takes the next wave in launch
order.  Prints the makespan over the mean SIMD work for the launch order,
for wave rounds taken in reverse (SF_TABLE_SNAKE) and for a greedy balanced
first round."""
import heapq
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from table_trace_report import load  # noqa: E402

S, D = 1024, 3


def makespan(L, order):
    n = len(L)
    fin = np.zeros(S)
    ev = []
    for w in range(min(n, S * D)):
        i = w % S
        fin[i] += L[order[w]]
        heapq.heappush(ev, (fin[i], i))
    for w in range(S * D, n):
        _, i = heapq.heappop(ev)
        fin[i] += L[order[w]]
        heapq.heappush(ev, (fin[i], i))
    return fin.max() / (L.sum() / S)


def reversed_rounds(n, rounds):
    o = list(range(n))
    for r in rounds:
        seg = list(range(r * S, min((r + 1) * S, n)))
        o[r * S:r * S + len(seg)] = seg[::-1]
    return o


def greedy_first_round(L):
    n = len(L)
    o = list(range(n))
    load, cnt, slots = np.zeros(S), np.zeros(S, int), {}
    for g in range(min(n, S * D)):
        cand = np.where(cnt < D)[0]
        i = cand[np.argmin(load[cand])]
        slots.setdefault(i, []).append(g)
        load[i] += L[g]
        cnt[i] += 1
    for i, gs in slots.items():
        for r, g in enumerate(gs):
            o[r * S + i] = g
    return o


def main():
    path = sys.argv[1]
    lst = sys.argv[2] if len(sys.argv) > 2 else "cdc"
    _s, _e, _key, nch, _nv = load(path, lst)
    L = nch.astype(float)
    n = len(L)
    print(f"{path} [{lst}]: {n} groups, makespan / mean SIMD work")
    print(f"  launch order            {makespan(L, list(range(n))):.4f}")
    for rounds in ([1], [2], [1, 2], [1, 3], [1, 2, 3]):
        print(f"  rounds {str(rounds):15s}  {makespan(L, reversed_rounds(n, rounds)):.4f}")
    print(f"  greedy first round      {makespan(L, greedy_first_round(L)):.4f}")


if __name__ == "__main__":
    main()
