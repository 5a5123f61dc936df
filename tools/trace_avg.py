"""Average duration of one kernel family over the timed steps of a
rocprofv3 --kernel-trace run (cross-check of bench.py's HIP-event roofline):

  python tools/trace_avg.py <trace_dir> <warmup> <name_regex>"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(f"{sys.argv[1]}/run_kernel_trace.csv")), key=lambda r: int(r["Dispatch_Id"]))
warmup, rx = int(sys.argv[2]), re.compile(sys.argv[3])
adam, durs, spans = 0, [], []
for n, r in enumerate(rows):
    if re.search(r"adamw(_dev)?_kernel", r["Kernel_Name"]):
        adam += 1
        continue
    if adam >= warmup and rx.search(r["Kernel_Name"]):
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        durs.append(t1 - t0)
        # the split-K / row-sum reduces launched by the same gemm call (bench.py's event window)
        m = n + 1
        while m < len(rows) and ("splitk_reduce" in rows[m]["Kernel_Name"] or "rowsum_reduce" in rows[m]["Kernel_Name"]):
            t1 = int(rows[m]["End_Timestamp"])
            m += 1
        spans.append(t1 - t0)
print(f"{len(durs)} launches after warm-up step {warmup}: GEMM kernel avg {sum(durs) / len(durs) / 1e3:.2f} us; "
      f"with its split-K reduce (bench.py event window) avg {sum(spans) / len(spans) / 1e3:.2f} us")
