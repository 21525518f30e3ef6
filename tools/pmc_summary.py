"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel (mean per dispatch)."""
import csv
import sys
from collections import defaultdict

f = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:40]
    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: f"{sum(v) / len(v):.4g}" for c, v in d.items()})
