"""Dev helper: sum rocprofv3 PMC counters of the POA kernel from a counter_collection.csv."""
import csv, sys
from collections import defaultdict
agg = defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if 'poa_kernel' in r['Kernel_Name']:
        agg[r['Counter_Name']] += float(r['Counter_Value'])
for k, v in sorted(agg.items()):
    print(f"{k:28s} {v:.4e}")
