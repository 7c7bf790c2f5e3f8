"""Average rocprofv3 --pmc counters per kernel (name filter) over the dispatches of one or more pass directories.
    python tools/kernel_pmc.py FILTER DIR [DIR ...]"""
import csv
import glob
import re
import sys
from collections import defaultdict


def main():
    filt, dirs = sys.argv[1], sys.argv[2:]
    tot = defaultdict(float)
    disp = defaultdict(set)
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for row in csv.DictReader(open(f)):
                name = re.sub(r"\(anonymous namespace\)::", "", row["Kernel_Name"])
                if not re.search(filt, name):
                    continue
                key = (re.sub(r"\(.*$", "", name)[:60], row["Counter_Name"])
                tot[key] += float(row["Counter_Value"])
                disp[key].add(row.get("Dispatch_Id", row.get("Correlation_Id")))
    for (k, c), v in sorted(tot.items()):
        n = max(1, len(disp[(k, c)]))
        print(f"{k:60s} {c:28s} {v / n:16.1f}  (x{n})")


if __name__ == "__main__":
    main()
