"""Average PMC counters per kernel name from rocprofv3 --pmc csv output dirs (counter_collection.csv)."""
import csv
import glob
import os
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name", r.get("Kernel-Name", "?"))
                acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, ctrs in acc.items():
    if "igemm" not in name and "bn_" not in name and "f32" not in name:
        continue
    print(name[:120])
    for k, v in sorted(ctrs.items()):
        print(f"   {k:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
