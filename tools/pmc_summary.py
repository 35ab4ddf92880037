"""Median per-dispatch PMC values of every counter_collection.csv under a dir."""
import csv
import statistics
import sys
from collections import defaultdict
from pathlib import Path

vals = defaultdict(list)
for f in sorted(Path(sys.argv[1]).rglob("*counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        vals[(row["Kernel_Name"][:60], row["Counter_Name"])].append(float(row["Counter_Value"]))
for (k, c), v in sorted(vals.items()):
    print(f"{k:60s} {c:28s} median {statistics.median(v):14.0f}  n={len(v)}")
