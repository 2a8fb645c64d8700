"""Summarise rocprofv3 --pmc counter_collection.csv files per kernel.

usage: python tools/pmcsum.py gpurun_out/pmc [substr ...]

Prints, per kernel name (optionally filtered by substrings), the number of
dispatches and the per-dispatch mean of every counter collected across the
passes, plus derived ratios when their inputs are present:
  wait%   = SQ_WAIT_ANY / SQ_WAVE_CYCLES          (parked on s_waitcnt / barrier)
  stall%  = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES     (issue stalls: MFMA RAW, pipe busy)
  active% = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  mfma%   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
            (busy cycles are summed over every SIMD; GRBM_GUI_ACTIVE over the 8 XCDs,
            MI355X_MICROARCH.md "SQ PMC units" / "DVFS give-back")
  ldsconf% = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
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


def derived(mean):
    """MFMA utilisation and LDS bank-conflict rate from per-dispatch means (None if absent)."""
    out = {}
    if mean.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None and mean.get("GRBM_GUI_ACTIVE"):
        out["mfma_util"] = mean["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * mean["GRBM_GUI_ACTIVE"] / 8.0)
    if mean.get("SQ_LDS_BANK_CONFLICT") is not None and mean.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_conflict_rate"] = mean["SQ_LDS_BANK_CONFLICT"] / mean["SQ_LDS_IDX_ACTIVE"]
    wc = mean.get("SQ_WAVE_CYCLES")
    if wc:
        for c, lab in (("SQ_WAIT_ANY", "wait"), ("SQ_WAIT_INST_ANY", "stall"), ("SQ_ACTIVE_INST_ANY", "active")):
            if c in mean:
                out[lab] = mean[c] / wc
    return out


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
        dv = derived(mean)
        if dv:
            print("   " + "  ".join(f"{k}={100 * v:.1f}%" for k, v in dv.items()))


if __name__ == "__main__":
    main()
