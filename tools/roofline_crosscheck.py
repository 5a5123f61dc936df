"""Cross-check the bench line's roofline kernel timing against the rocprofv3 kernel trace of the
same run (tools/prof_traffic.sh writes both: <tag>_trace/run_kernel_trace.csv and <tag>_trace.log).

  python tools/roofline_crosscheck.py <trace_dir> <bench_log> <warmup_steps> [default_bench_json]

The line's `roofline.kernel_regex` names the family (e.g. `gemm_f32<0, 0, 0, 0>`: the fp32
kernels gemm_f32_kernel<0, 0, 0, 0, ...> and gemm_glds_kernel<0, 0, ...>); the trace's launches
of that family after the warm-up steps (a step ends at the AdamW dispatch) are averaged and set
beside the HIP-event average the line reports.  Also prints the runner-up family, since the two
largest fp32 families are within a percent of each other on the NYU step."""
import csv
import json
import re
import sys


def family_of(name):
    m = re.search(r"gemm_f32_kernel<(\d+), (\d+), (\d+), (\d+),", name)
    if m:
        return "gemm_f32<{}, {}, {}, {}>".format(*m.groups())
    m = re.search(r"gemm_glds_kernel<(\d+), (\d+),", name)
    if m:
        return "gemm_f32<{}, {}, 0, 0>".format(*m.groups())
    m = re.search(r"gemm_b16_kernel<(\d+), (\d+),", name)
    if m:
        return "gemm_b16_kernel<{}, {},".format(*m.groups())
    return None


def main():
    tdir, blog, warm = sys.argv[1], sys.argv[2], int(sys.argv[3])
    line = [ln for ln in open(blog) if ln.startswith('{"metric')][-1]
    d = json.loads(line)
    rf = d["roofline"]
    rows = sorted(csv.DictReader(open(f"{tdir}/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
    adam, fam, red, last = 0, {}, {}, None
    for r in rows:
        n = r["Kernel_Name"]
        if re.search(r"adamw(_dev)?_kernel", n):
            adam += 1
            continue
        if adam < warm:
            continue
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        f = family_of(n)
        if f:
            fam.setdefault(f, []).append(dur)
            red.setdefault(f, []).append(0.0)
            last = f
        elif "gemm_splitk_reduce" in n and last is not None:  # inside the same entry-point call
            red[last][-1] += dur
        else:
            last = None
    steps = adam - warm
    key = rf["kernel_regex"]
    t = fam.get(key, [])
    tot = sorted(((sum(v), k) for k, v in fam.items()), reverse=True)
    print(f"{d['config']['workload']} (bench.py under rocprofv3 --kernel-trace, {steps} timed steps after {warm} "
          f"warm-up)")
    print(f"dominant family in the line: {key} ({rf['kernel']}), {len(t) / max(steps, 1):.1f} launches/step")
    if t:
        avg = sum(t) / len(t)
        avg2 = avg + sum(red.get(key, [])) / len(t)
        if rf["unit"] == "TFLOP/s":
            rate = lambda us: f"{rf['flops_per_launch'] / us / 1e6:.2f} TF/s = {rf['flops_per_launch'] / us / 1e6 / rf['peak']:.4f} of {rf['peak']}"  # noqa: E731
        else:
            rate = lambda us: f"{rf['algorithmic_bytes'] / us / 1e3:.1f} GB/s = {rf['algorithmic_bytes'] / us / 1e3 / rf['peak']:.4f} of {rf['peak']}"  # noqa: E731
        print(f"rocprofv3 trace: average {avg:.2f} us per GEMM kernel -> {rate(avg)}")
        print(f"  with the split-K reduce kernels the same entry-point calls launch (what the events "
              f"bracket): {avg2:.2f} us -> {rate(avg2)}")
    print(f"bench HIP events (same run): {rf['avg_launch_us']} us per launch -> frac {rf['frac']} ({rf['achieved']} "
          f"{rf['unit']})")
    print("families by trace time per step (ms): " + ", ".join(f"{k} {s / max(steps, 1) / 1e3:.2f}" for s, k in tot[:4]))
    if len(tot) > 1:
        print(f"the top two families differ by {100 * (tot[0][0] - tot[1][0]) / tot[0][0]:.1f} % of trace time: "
              "the line names whichever its instrumented step measures larger")
    if len(sys.argv) > 4:
        dd = json.loads([ln for ln in open(sys.argv[4]) if ln.startswith('{"metric')][-1])
        r2 = dd["roofline"]
        print(f"default bench line (no profiler, {sys.argv[4]}): {r2['kernel_regex']} frac {r2['frac']}, "
              f"{r2['achieved']} TF/s, {r2['avg_launch_us']} us per launch")


if __name__ == "__main__":
    main()
