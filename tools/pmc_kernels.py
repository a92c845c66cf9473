"""Mean of every counter per kernel name (one rocprofv3 --pmc counter_collection.csv)."""
import csv
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    acc[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, cs in acc.items():
    print(n[:80], len(next(iter(cs.values()))), {c: round(sum(v) / len(v)) for c, v in cs.items()})
