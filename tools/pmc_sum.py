"""Sum rocprofv3 --pmc counters per kernel (first 60 chars of the name)."""
import csv, collections, sys
for path in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        agg[r['Kernel_Name'][:60]][r['Counter_Name']] += float(r['Counter_Value'])
    for k, v in agg.items():
        if 'rocclr' in k or 'elementwise' in k:
            continue
        print(k)
        print("  " + " ".join(f"{a}={b:.4g}" for a, b in sorted(v.items())))
