#!/usr/bin/env python3
"""Cross-XCD counter litmus (sf_test_xcd_litmus, syncfast_amd/csrc/sf_litmus.hip).

Runs `--trials` launches of each read form, alternating, and prints one JSON
line per launch and a summary: how often the second read of a counter that
other XCDs added to after the reader's XCD L2 took its line returned the
stale first value.  mode 0 = relaxed agent-scope atomic load (the fused
launch's poll until round 6), mode 1 = agent-scope add of an opaque zero (the
poll now).  Evidence for DESIGN.md 3.3."""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=50)
    a = ap.parse_args()
    import torch
    from syncfast_amd._lib import lib
    torch.cuda.set_device(0)
    summary = {0: {"launches": 0, "stale": 0, "partial": 0, "exact": 0, "bad": 0},
               1: {"launches": 0, "stale": 0, "partial": 0, "exact": 0, "bad": 0}}
    for t in range(a.trials):
        for mode in (0, 1) if t % 2 == 0 else (1, 0):
            out = (ctypes.c_uint32 * 8)()
            rc = lib().sf_test_xcd_litmus(mode, out)
            status, xcc, adders, v0, v1, fresh = list(out)[:6]
            s = summary[mode]
            s["launches"] += 1
            if rc != 0 or status != 0 or fresh != adders:
                s["bad"] += 1
            elif v1 == v0:
                s["stale"] += 1
            elif v1 == adders:
                s["exact"] += 1
            else:
                s["partial"] += 1
            print(json.dumps({"trial": t, "mode": mode, "rc": rc, "status": status, "reader_xcc": xcc,
                              "adds_other_xcds": adders, "first_read": v0, "second_read": v1,
                              "rmw_read_after": fresh}), flush=True)
    print(json.dumps({"summary": {("load" if m == 0 else "rmw"): v for m, v in summary.items()}}), flush=True)


if __name__ == "__main__":
    main()
