"""Average PMC counters per kernel from rocprofv3 csv passes."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"][:60]
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        # each dispatch reports one value per counter (summed over dims by rocprofv3)
        print(f"   {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
