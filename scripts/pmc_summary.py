"""Summarise scripts/pmc.sh output per kernel: mean counter value per dispatch.
usage: python scripts/pmc_summary.py <tag> [--json out.json]"""
import csv
import glob
import json
import sys
from collections import defaultdict

tag = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"gpurun_out/pmc_{tag}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
summary = {}
for k, d in acc.items():
    summary[k] = {c: sum(v) / len(v) for c, v in d.items()}
    print(k[:90])
    for c, v in sorted(summary[k].items()):
        print(f"   {c:28s} {v:.4g}")
try:  # the build the passes ran (scripts/pmc.sh wrote it): bench.py ignores counters of another build
    summary["__build__"] = {"lib_sha256": open(f"gpurun_out/pmc_{tag}/lib_sha256.txt").read().strip(),
                            "tag": tag}
except OSError:
    pass
if "--json" in sys.argv:
    out = sys.argv[sys.argv.index("--json") + 1]
    json.dump(summary, open(out, "w"), indent=1, sort_keys=True)
