"""Per-kernel sums of rocprofv3 --pmc counters (counter_collection.csv files under a directory)."""
import csv
import glob
import sys
from collections import defaultdict

tot = defaultdict(lambda: defaultdict(float))
calls = defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:48]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
names = sorted({c for v in tot.values() for c in v})
print("| kernel | dispatches | " + " | ".join(names) + " |")
print("|---|---|" + "---|" * len(names))
for k, v in sorted(tot.items(), key=lambda kv: -max(kv[1].values())):
    print(f"| `{k}` | {len(calls[k])} | " + " | ".join(f"{v.get(n, 0):.3g}" for n in names) + " |")
