"""Print the kernel sequence of the last complete learner iteration of a
rocprofv3 kernel trace (tools/gpu_prof.sh): start offset, duration, name.

usage: python tools/prof_iter.py gpurun_out/prof_c3 [first-kernel-substring]"""
import csv
import re
import sys

d = sys.argv[1]
mark = sys.argv[2] if len(sys.argv) > 2 else None
r = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
r.sort(key=lambda x: int(x["Start_Timestamp"]))
names = [x["Kernel_Name"] for x in r]
if mark is None:   # the iteration's first kernel: the frame encoder or the frame layout pass
    mark = next(m for m in ("k_vision_fwd", "k_frames_rgbx") if any(m in n for n in names))
idx = [i for i, n in enumerate(names) if mark in n]
s, e = idx[-2], idx[-1]
t0 = int(r[s]["Start_Timestamp"])
tot = 0.0
for x in r[s:e]:
    dur = (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3
    tot += dur
    n = re.sub(r"_ZN3aaa|aaa::", "", x["Kernel_Name"])[:110]
    print(f"{(int(x['Start_Timestamp']) - t0) / 1e3:9.1f} {dur:8.1f}  {n}")
print(f"iteration span {(int(r[e]['Start_Timestamp']) - t0) / 1e3:.1f} us, kernel sum {tot:.1f} us")
