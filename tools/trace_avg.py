"""Average duration of one kernel family over the timed steps of a
rocprofv3 --kernel-trace run (cross-check of bench.py's HIP-event roofline):

  python tools/trace_avg.py <trace_dir> <warmup> <name_regex>"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(f"{sys.argv[1]}/run_kernel_trace.csv")), key=lambda r: int(r["Dispatch_Id"]))
warmup, rx = int(sys.argv[2]), re.compile(sys.argv[3])
adam, durs, steps = 0, [], []
for r in rows:
    if "adamw_kernel" in r["Kernel_Name"]:
        adam += 1
        continue
    if adam >= warmup and rx.search(r["Kernel_Name"]):
        durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
print(f"{len(durs)} launches after warm-up step {warmup}: avg {sum(durs) / len(durs) / 1e3:.2f} us")
