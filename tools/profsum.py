import csv, sys
rows = list(csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_stats.csv")))
it = 7
tot = sum(float(r["TotalDurationNs"]) for r in rows) / 1e6 / it
print(f"total GPU time per iteration {tot:.3f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 24]:
    n = r["Name"]
    short = n.replace("aaa::", "").replace("float", "f").replace("GemmCfg", "G")[:120]
    print(f'{float(r["TotalDurationNs"])/1e6/it:8.3f} ms/it calls {int(r["Calls"])/it:5.1f}/it avg {float(r["AverageNs"])/1e3:8.2f} us  {short}')
