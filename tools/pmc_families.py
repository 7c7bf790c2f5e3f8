"""Per-family HBM traffic and MFMA busy of the training step from rocprofv3 PMC passes -> profiles/pmc_<key>.json.

    python tools/pmc_families.py KEY STEPS OUT.json PASS_DIR [PASS_DIR ...]

Each PASS_DIR holds one `rocprofv3 --pmc ... --output-format csv` run of `bench.py --steps STEPS --warmup W
--no-roofline --no-cpu-baseline --no-gemm-peak` (one counter group per pass: FETCH_SIZE | WRITE_SIZE | SQ group |
GRBM_GUI_ACTIVE).  Dispatches are summed per kernel name over the whole run and divided by (STEPS + W) — the bench
runs W + STEPS identical steps — and kernels are grouped into the families bench.py times live:

  gemm_wgrad  gemm_bf16_v4<false, false, float, 4> + splitk_reduce_kernel<float>   (weight gradients, split-K)
  gemm_fwd    gemm_bf16_v4<true, true, ...>                                        (forward Linears, patch embed)
  gemm_dgrad  gemm_bf16_v4<true, false, ...>                                       (input gradients)
  attn_fwd / attn_bwd / ln_fwd / ln_bwd, and `other`.

FETCH_SIZE is doubled (gfx950 reports half of the bytes of 16-B/lane streaming reads, MI355X_MICROARCH.md §HBM);
WRITE_SIZE is taken as reported (exact for 16-B/lane stores).  Both are KiB in rocprofv3's csv."""
import csv
import glob
import json
import os
import re
import sys


def family(name):
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    if "splitk_reduce_kernel<float>" in n or re.search(r"gemm_bf16_v4<false, false", n):
        return "gemm_wgrad"
    if re.search(r"gemm_bf16_v4<true, true", n):
        return "gemm_fwd"
    if re.search(r"gemm_bf16_v4<true, false", n):
        return "gemm_dgrad"
    if "splitk_reduce_kernel<unsigned short>" in n:
        return "gemm_tail_reduce"
    if "attn_fwd" in n:
        return "attn_fwd"
    if "attn_bwd" in n or "attn_delta" in n:
        return "attn_bwd"
    if "ln_fwd" in n:
        return "ln_fwd"
    if "ln_bwd" in n:
        return "ln_bwd"
    return "other"


def short(name):
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = re.sub(r"^void ", "", n)
    return re.sub(r"\((?!anonymous).*$", "", n)[:90]


def derived(cs):
    d = {}
    if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
        rd, wr = 2 * cs["FETCH_SIZE"] * 1024, cs["WRITE_SIZE"] * 1024
        d.update(hbm_read_bytes_per_step=int(rd), hbm_write_bytes_per_step=int(wr), hbm_bytes_per_step=int(rd + wr))
    if "SQ_VALU_MFMA_BUSY_CYCLES" in cs and "GRBM_GUI_ACTIVE" in cs:
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs: active GPU cycles = GRBM / 8; 1024 SIMDs
        d["mfma_busy_frac"] = round(cs["SQ_VALU_MFMA_BUSY_CYCLES"] * 8 / (1024 * cs["GRBM_GUI_ACTIVE"]), 4)
    if "SQ_WAIT_ANY" in cs and "SQ_WAVE_CYCLES" in cs:
        d["wave_frac_parked_waitcnt_barrier"] = round(cs["SQ_WAIT_ANY"] / cs["SQ_WAVE_CYCLES"], 4)
    if "SQ_WAIT_INST_ANY" in cs and "SQ_WAVE_CYCLES" in cs:
        d["wave_frac_issue_stalled"] = round(cs["SQ_WAIT_INST_ANY"] / cs["SQ_WAVE_CYCLES"], 4)
    return d


def load(dirs):
    """{counter: {kernel: value summed over its dispatches}}"""
    vals = {}
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                k, c, v = r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"])
                vals.setdefault(c, {}).setdefault(k, 0.0)
                vals[c][k] += v
    return vals


def main():
    key, steps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    vals = load(sys.argv[4:])
    fams, kers = {}, {}
    for c, per in vals.items():
        for k, v in per.items():
            f = fams.setdefault(family(k), {})
            f[c] = f.get(c, 0.0) + v / steps
            kk = kers.setdefault(short(k), {})
            kk[c] = kk.get(c, 0.0) + v / steps
    res = {f: dict(counters_per_step={c: round(v, 1) for c, v in sorted(cs.items())}, **derived(cs))
           for f, cs in fams.items()}
    kres = {k: dict(family=family(k), **derived(cs)) for k, cs in kers.items()}
    kres = dict(sorted(kres.items(), key=lambda kv: -kv[1].get("hbm_bytes_per_step", 0)))
    sargs = os.environ.get("PMC_SCHEDULE_ARGS", "").strip()
    json.dump({"workload_key": key, "steps_divisor": steps,
               "schedule": ("in-order (" + sargs + "): the schedule of bench.py's event-bracketed roofline step")
               if sargs else "default (two forward chains + weight-gradient stream)",
               "method": "rocprofv3 --pmc, one counter group per pass over bench.py; per-kernel sums / steps; "
                         "FETCH_SIZE x2 (gfx950), WRITE_SIZE as reported; KiB -> bytes",
               "families": res, "kernels": kres}, open(out, "w"), indent=1)
    print(json.dumps({f: {k: v for k, v in d.items() if k != "counters_per_step"} for f, d in res.items()}, indent=1))
    for k, d in list(kres.items())[:16]:
        print(f"{d.get('hbm_bytes_per_step', 0) / 1e6:9.1f} MB/step  mfma {d.get('mfma_busy_frac', 0):.3f}  {k}")


if __name__ == "__main__":
    main()
