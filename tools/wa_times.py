"""Average duration per (kernel, grid) of the window-attention kernels in a rocprofv3 kernel trace."""
import collections
import csv
import sys

d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "winattn_fwd" in n or "winattn_bwd_kernel" in n:
        d[(n.split("(")[0].replace("void mdemi::", ""), int(r["Grid_Size_X"]))].append(
            int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(d.items()):
    print(f"{k[0]:32s} grid {k[1]:8d} x{len(v):3d} {sum(v) / len(v) / 1e3:8.1f} us")
