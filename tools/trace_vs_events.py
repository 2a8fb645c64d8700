"""Reconcile bench.py's HIP-event kernel times with a rocprofv3 kernel trace of
the SAME process.

  rocprofv3 --kernel-trace --stats -d D -o run --output-format csv -- \
      python bench.py --timed-steps K ... > bench.json
  python tools/trace_vs_events.py D/run_kernel_trace.csv bench.json K

For every MFMA timer class of the bench line (forward recurrence, BPTT,
ConvLSTM weight gradient) the dispatched kernel is named by the variant's
``[kernel: a+b]`` marker; the trace's launches of that kernel are taken in
dispatch order, the last K * launches-per-step of them are the timed steps'
launches, and their mean duration is set beside the events' mean.  Also prints
the whole run's launch-by-launch trend of the dominant kernel (the r04 traces
were taken over 7 launches of a --steps 5 --warmup 2 run, still on the clock /
first-touch ramp).
"""
import csv
import json
import re
import sys


def main():
    trace, bench = sys.argv[1], sys.argv[2]
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    line = json.loads(open(bench).read().strip().splitlines()[-1])
    out = {"trace": trace, "bench": bench, "timed_steps": K, "classes": {}}
    for name, k in line["kernels"].items():
        if "avg_us" not in k:
            continue
        m = re.search(r"\[kernel: ([^\]]+)\]", k.get("variant", ""))
        if not m:
            continue
        subs = m.group(1).split("+")
        hits = [r for r in rows if all(s in r["Kernel_Name"] for s in subs)]
        per_step = max(1, k["launches"] // K)
        last = hits[-K * per_step:]
        durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in last]
        alld = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in hits]
        mean = sum(durs) / max(len(durs), 1)
        out["classes"][name] = {
            "kernel": last[-1]["Kernel_Name"][:120] if last else None,
            "event_avg_us": k["avg_us"], "trace_avg_us_timed": round(mean, 2),
            "trace_last_us": round(durs[-1], 2) if durs else None,
            "ratio_trace_over_event": round(mean / k["avg_us"], 4) if durs else None,
            "launches_in_trace": len(hits),
            "trend_us": [round(d, 1) for d in alld],
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
