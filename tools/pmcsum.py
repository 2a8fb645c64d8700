"""Summarise rocprofv3 --pmc counter_collection.csv files per kernel.

usage: python tools/pmcsum.py gpurun_out/pmc [substr ...]

Prints, per kernel name (optionally filtered by substrings), the number of
dispatches and the per-dispatch mean of every counter collected across the
passes, plus derived ratios when their inputs are present:
  wait%   = SQ_WAIT_ANY / SQ_WAVE_CYCLES          (parked on s_waitcnt / barrier)
  stall%  = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES     (issue stalls: MFMA RAW, pipe busy)
  active% = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  FETCH_SIZE / WRITE_SIZE are KB per dispatch (rocprofv3 unit) -> MB shown.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    acc = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [values per dispatch]
    for f in sorted(glob.glob(os.path.join(d, "*counter_collection.csv"))):
        per = defaultdict(float)   # (dispatch, kernel, counter) -> value summed over XCD rows
        for row in csv.DictReader(open(f)):
            per[(row["Dispatch_Id"], row["Kernel_Name"], row["Counter_Name"])] += float(row["Counter_Value"])
        for (disp, k, c), v in per.items():
            acc[k][c].append(v)
    return acc


def short(k):
    return k if len(k) < 110 else k[:107] + "..."


def main():
    d = sys.argv[1]
    subs = sys.argv[2:]
    acc = load(d)
    for k, cs in sorted(acc.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0]))):
        if subs and not any(s in k for s in subs):
            continue
        n = max(len(v) for v in cs.values())
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        print(f"{short(k)}  dispatches={n}")
        line = []
        for c in sorted(mean):
            v = mean[c]
            if c in ("FETCH_SIZE", "WRITE_SIZE"):
                line.append(f"{c}={v / 1024:.2f}MB")
            else:
                line.append(f"{c}={v:.4g}")
        print("   " + "  ".join(line))
        wc = mean.get("SQ_WAVE_CYCLES")
        if wc:
            parts = []
            for c, lab in (("SQ_WAIT_ANY", "wait"), ("SQ_WAIT_INST_ANY", "stall"), ("SQ_ACTIVE_INST_ANY", "active")):
                if c in mean:
                    parts.append(f"{lab}={100 * mean[c] / wc:.1f}%")
            if parts:
                print("   " + "  ".join(parts))


if __name__ == "__main__":
    main()
