#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs per kernel: average counter value per dispatch."""
import csv
import glob
import json
import sys
from collections import defaultdict

out = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{out}/pass*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        full = r["Kernel_Name"].split("(")[0].strip()   # (template arguments kept: instances apart)
        name = full.split("<")[0].split("::")[-1] + full[len(full.split("<")[0]):]
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
summary = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}
print(json.dumps(summary, indent=1))
