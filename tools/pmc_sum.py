"""Dev helper: sum rocprofv3 PMC counters of the POA kernel over counter_collection.csv files
(arguments: csv files or directories searched recursively; KERNEL=<substring> picks another kernel)."""
import csv, os, sys
from collections import defaultdict
agg = defaultdict(float)
paths = []
for a in sys.argv[1:]:
    if os.path.isdir(a):
        for root, _, files in os.walk(a):
            paths += [os.path.join(root, f) for f in files if f.endswith("counter_collection.csv")]
    else:
        paths.append(a)
for p in paths:
    for r in csv.DictReader(open(p)):
        if os.environ.get('KERNEL', 'poa_kernel') in r['Kernel_Name']:
            agg[r['Counter_Name']] += float(r['Counter_Value'])
for k, v in sorted(agg.items()):
    print(f"{k:28s} {v:.4e}")
