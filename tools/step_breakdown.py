"""Per-kernel time per TIMED train step from a rocprofv3 --kernel-trace run of bench.py
(steps are delimited by the single adamw_kernel dispatch that ends each one; the warm-up
steps, which include the GEMM autotuning, are skipped):

  python tools/step_breakdown.py <trace_dir> <warmup> [top] [--by-grid]

Reports wall vs kernel-busy time per step, per-family totals and the top kernels
(--by-grid: GEMM kernels keyed by name and grid size, i.e. per output-tile x split shape)."""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(f"{sys.argv[1]}/run_kernel_trace.csv")), key=lambda r: int(r["Dispatch_Id"]))
by_grid = "--by-grid" in sys.argv
argv = [a for a in sys.argv if a != "--by-grid"]
warmup = int(argv[2])
top = int(argv[3]) if len(argv) > 3 else 40
adam_idx = [i for i, r in enumerate(rows) if re.search(r"adamw(_dev)?_kernel", r["Kernel_Name"])]
lo, hi = adam_idx[warmup - 1] + 1, adam_idx[-1] + 1
steps = len(adam_idx) - warmup
win = rows[lo:hi]
by = collections.defaultdict(lambda: [0, 0])
busy = 0
for r in win:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    name = re.sub(r"\(.*", "", r["Kernel_Name"])
    name = re.sub(r"^void ", "", name)
    if by_grid and "gemm_" in name:
        name = f"{name} grid {int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])}"
    by[name][0] += d
    by[name][1] += 1
    busy += d
span = int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])
print(f"{steps} timed steps: wall {span / steps / 1e6:.2f} ms/step, kernel busy {busy / steps / 1e6:.2f} ms/step, "
      f"{len(win) / steps:.0f} launches/step")
fam = collections.defaultdict(float)
for name, (d, n) in by.items():
    key = "gemm" if any(g in name for g in ("gemm_f32_kernel", "gemm_glds_kernel", "gemm_m16_kernel", "gemm_b16_kernel")) else ("winattn" if "winattn" in name else name)
    fam[key] += d
print("families (ms/step):", ", ".join(f"{k} {v / steps / 1e6:.2f}"
                                       for k, v in sorted(fam.items(), key=lambda kv: -kv[1])[:14]))
for name, (d, n) in sorted(by.items(), key=lambda kv: -kv[1][0])[:top]:
    print(f"{d / steps / 1e6:8.2f} ms/step {n / steps:7.1f}/step {d / n / 1e3:9.1f} us  {name[:100]}")
