"""Summarise scripts/pmc.sh output per kernel: mean counter value per dispatch."""
import csv
import glob
import sys
from collections import defaultdict

tag = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"gpurun_out/pmc_{tag}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")[:60]
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v) / len(v):.4g}  (n={len(v)})")
