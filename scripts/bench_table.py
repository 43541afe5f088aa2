"""Markdown table of the bench lines in a profiles directory (value, step, dominant kernel, roofline).
usage: python scripts/bench_table.py profiles/r4"""
import glob
import json
import os
import sys

d = sys.argv[1]
print("| line | value | unit | ms/step | kernel | kernel ms | bound | frac | traffic/launch | cpu baseline |")
print("|---|---|---|---|---|---|---|---|---|---|")
for f in sorted(glob.glob(os.path.join(d, "bench_*.json"))):
    try:
        line = [l for l in open(f).read().splitlines() if l.startswith("{")][-1]
        j = json.loads(line)
    except (IndexError, ValueError):
        continue
    r = j.get("roofline") or {}
    cb = j.get("cpu_baseline") or {}
    tr = r.get("traffic")
    cpu = f"{cb['value']:.3g} ({cb.get('cores')} thr)" if cb.get("value") else "-"
    print(f"| {os.path.basename(f)[6:-5]} | {j['value']:.4g} | {j['unit']} | {j['ms_per_step']:.4f} | "
          f"`{str(r.get('kernel', ''))[:48]}` | {r.get('kernel_ms') or 0:.4f} | {r.get('bound')} | "
          f"{r.get('frac') or 0:.3f} | {'%.3g B' % tr if tr else '-'} | {cpu} |")
