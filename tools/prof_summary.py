"""Markdown table from a rocprofv3 --stats kernel_stats.csv:  python tools/prof_summary.py STATS.csv STEPS TITLE"""
import csv
import re
import sys

path, steps, title = sys.argv[1], int(sys.argv[2]), sys.argv[3]
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"# {title}\n")
print("| kernel | calls | total ms | ms/step | avg us | share |\n|---|---|---|---|---|---|")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    t = float(r["TotalDurationNs"])
    if t / tot < 0.0005:
        continue
    name = re.sub(r"\(anonymous namespace\)::", "", r["Name"])
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\((?!anonymous).*$", "", name)[:80]
    print(f"| `{name}` | {r['Calls']} | {t/1e6:.2f} | {t/1e6/steps:.2f} | {float(r['AverageNs'])/1e3:.1f} | "
          f"{100*t/tot:.1f}% |")
print(f"\nTotal kernel time {tot/1e6:.1f} ms over {steps} steps = {tot/1e6/steps:.1f} ms/step of GPU kernel time.")
