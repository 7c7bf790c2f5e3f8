"""Per-step kernel table of the TIMED steps only, from a rocprofv3 --kernel-trace run of bench.py.

    python tools/prof_steps.py KERNEL_TRACE.csv WARMUP STEPS TITLE [BENCH_JSON]

bench.py runs WARMUP + STEPS identical training steps; each ends with exactly one `adamw_kernel` launch.  Dispatches
are ordered by start time and cut after the WARMUP-th adamw_kernel (warmup, one-time optimizer-state fills and the
first-step table uploads fall before the cut) and after the last one (the measured GEMM peak and anything else bench.py
runs after the timed loop fall after it).  The table sums kernel durations per name over the STEPS timed steps; the
footer compares the per-step kernel-time sum with bench.py's ms_per_step when its JSON line is given."""
import csv
import json
import re
import sys


def short(name):
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = re.sub(r"^void ", "", n)
    return re.sub(r"\((?!anonymous).*$", "", n)[:90]


def main():
    path, warm, steps, title = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    rows = list(csv.DictReader(open(path)))
    key_s = "Start_Timestamp" if "Start_Timestamp" in rows[0] else "start"
    key_e = "End_Timestamp" if "End_Timestamp" in rows[0] else "end"
    key_n = "Kernel_Name" if "Kernel_Name" in rows[0] else "name"
    rows.sort(key=lambda r: int(r[key_s]))
    ends = [i for i, r in enumerate(rows) if "adamw_kernel" in r[key_n]]
    if len(ends) != warm + steps:
        sys.exit(f"expected {warm + steps} adamw_kernel launches, found {len(ends)}")
    lo, hi = ends[warm - 1] + 1, ends[-1] + 1
    sel = rows[lo:hi]
    t0, t1 = int(sel[0][key_s]), int(sel[-1][key_e])
    agg = {}
    for r in sel:
        d = int(r[key_e]) - int(r[key_s])
        a = agg.setdefault(short(r[key_n]), [0, 0])
        a[0] += 1
        a[1] += d
    tot = sum(v[1] for v in agg.values())
    print(f"# {title}\n")
    print(f"Timed steps only: dispatches {lo}..{hi - 1} of {len(rows)} (after warmup adamw #{warm}, through the last "
          f"adamw), {steps} steps.\n")
    print("| kernel | calls/step | ms/step | avg us | share |\n|---|---|---|---|---|")
    for name, (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        if d / tot < 0.0005:
            continue
        print(f"| `{name}` | {n / steps:.1f} | {d / 1e6 / steps:.3f} | {d / n / 1e3:.1f} | {100 * d / tot:.1f}% |")
    per = tot / 1e6 / steps
    wall = (t1 - t0) / 1e6 / steps
    # union of the kernels' [start, end) intervals over every stream: the time at least one kernel runs
    iv = sorted((int(r[key_s]), int(r[key_e]), short(r[key_n])) for r in sel)
    busy, cs, ce, last = 0, iv[0][0], iv[0][1], iv[0][2]
    gaps = {}                                # (kernel that ended last, kernel that starts next) -> [ns, count]
    for s_, e_, n_ in iv[1:]:
        if s_ > ce:
            busy += ce - cs
            g = gaps.setdefault((last, n_), [0, 0])
            g[0] += s_ - ce
            g[1] += 1
            cs, ce, last = s_, e_, n_
        elif e_ > ce:
            ce, last = e_, n_
    busy += ce - cs
    busy_ms = busy / 1e6 / steps
    print(f"\nKernel time {per:.2f} ms/step; first-to-last dispatch wall {wall:.2f} ms/step "
          f"(gaps {100 * (wall - per) / wall:.1f}%).")
    print(f"At least one kernel running: {busy_ms:.2f} ms/step ({100 * busy_ms / wall:.1f}% of the wall); kernel time / "
          f"busy time = {per / busy_ms:.2f} (average kernels in flight while any runs).")
    print("\nIdle gaps (no kernel running), by the kernel that ended last and the one that started next, largest first:\n")
    print("| after | before | us/step | gaps/step |\n|---|---|---|---|")
    for (a, b), (ns, c) in sorted(gaps.items(), key=lambda kv: -kv[1][0])[:15]:
        print(f"| `{a[:48]}` | `{b[:48]}` | {ns / 1e3 / steps:.1f} | {c / steps:.1f} |")
    if len(sys.argv) > 5:
        try:
            b = json.loads(open(sys.argv[5]).read().strip().splitlines()[-1])
            print(f"bench.py under the profiler: {b['ms_per_step']:.2f} ms/step ({b['value']:.0f} img/s); kernel-time "
                  f"sum / bench step = {per / b['ms_per_step']:.3f}.")
        except (OSError, ValueError, KeyError, IndexError):
            pass


if __name__ == "__main__":
    main()
