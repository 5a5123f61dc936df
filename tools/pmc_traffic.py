"""HBM traffic per launch of each GEMM kernel family from rocprofv3 --pmc passes.

  python tools/pmc_traffic.py <fetch_dir> <write_dir> <warmup> <workload> <out.json> [source note]

FETCH_SIZE / WRITE_SIZE come from separate passes (they do not fit one TCC
pass on gfx950) and are reported in KB.  Per MI355X_MICROARCH.md (HBM
section) FETCH_SIZE counts exactly half the bytes of wide coalesced reads on
gfx950, so it is doubled; WRITE_SIZE is exact for 16-B stores.  Only the
timed steps count: a step ends with the single mdemi::adamw_kernel dispatch,
so dispatches after the `warmup`-th adamw are kept (this excludes the GEMM
autotuner's first-use timing launches).  Launches are grouped by the
template-argument prefix `gemm_f32_kernel<A, B, AOP, BOP,` that bench.py's
roofline names, so whichever family dominates a run finds its traffic.  The fp32 family's
two kernel templates -- register-staged gemm_f32_kernel<A, B, AOP, BOP, ...> and the
direct-to-LDS gemm_glds_kernel<A, B, ...> (no load-time op) -- are one family, keyed
`gemm_f32<A, B, AOP, BOP>`: the per-shape autotuner picks among them.  The bf16-operand
kernel (gemm_b16_kernel<AL, BL, BMT, OCC>, gemm_b16_kernel.h) is keyed by its
`gemm_b16_kernel<AL, BL,` prefix, covering both row-tile variants."""
import csv
import json
import re
import sys

FAMILY = re.compile(r"gemm_f32_kernel<\d+, \d+, \d+, \d+,|gemm_glds_kernel<\d+, \d+,|"
                    r"gemm_m16_kernel<\d+, \d+, \d+, \d+, \d+,|gemm_b16_kernel<\d+, \d+,|winattn_\w+_kernel|binhead_nhwc_\w+")
F32 = re.compile(r"gemm_f32_kernel<(\d+), (\d+), (\d+), (\d+),")
GLDS = re.compile(r"gemm_glds_kernel<(\d+), (\d+),")


def family_key(match):
    """Canonical family of a kernel-name match (see the module docstring)."""
    m = F32.match(match)
    if m:
        return "gemm_f32<{}, {}, {}, {}>".format(*m.groups())
    m = GLDS.match(match)
    if m:
        return "gemm_f32<{}, {}, 0, 0>".format(*m.groups())
    return match


def per_family(path, counter, warmup):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Dispatch_Id"]))
    seen_adam, vals = 0, {}
    for r in rows:
        name = r["Kernel_Name"]
        if re.search(r"adamw(_dev)?_kernel", name):
            seen_adam += 1
            continue
        m = FAMILY.search(name)
        if seen_adam >= warmup and m and r["Counter_Name"] == counter:
            vals.setdefault(family_key(m.group(0)), []).append(float(r["Counter_Value"]) * 1024.0)
    return vals


def main():
    fdir, wdir, warmup, workload, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4], sys.argv[5]
    note = sys.argv[6] if len(sys.argv) > 6 else ""
    f = per_family(f"{fdir}/run_counter_collection.csv", "FETCH_SIZE", warmup)
    w = per_family(f"{wdir}/run_counter_collection.csv", "WRITE_SIZE", warmup)
    fams = {}
    for rx in sorted(set(f) & set(w)):
        fb = 2.0 * sum(f[rx]) / len(f[rx])
        wb = sum(w[rx]) / len(w[rx])
        fams[rx] = {"launches_fetch": len(f[rx]), "launches_write": len(w[rx]),
                    "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                    "traffic_bytes_per_launch": fb + wb}
    try:
        prof = json.load(open(out))
    except (OSError, ValueError):
        prof = {}
    old = prof.get(workload, {}).get("families", {})
    old.update(fams)
    for k in [k for k in old if k.startswith("gemm_f32_kernel<")]:
        del old[k]  # pre-round-4 key form, superseded by the gemm_f32<...> family keys
    prof[workload] = {"families": old,
                      "correction": "FETCH_SIZE x2 (gfx950 half-count of 16-B coalesced reads); KB->bytes x1024",
                      "source": note}
    json.dump(prof, open(out, "w"), indent=1)
    print(json.dumps(prof[workload]))


if __name__ == "__main__":
    main()
