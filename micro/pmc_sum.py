"""Mean per launch of each PMC counter for the timed C4 search instance (k_knn_*<..., false...>) in a
rocprofv3 --pmc output directory. usage: python micro/pmc_sum.py DIR"""
import csv
import os
import re
import sys
from collections import defaultdict

vals = defaultdict(list)
for root, _, files in os.walk(sys.argv[1]):
    for f in files:
        if f.endswith("counter_collection.csv"):
            for r in csv.DictReader(open(os.path.join(root, f))):
                if re.search(r"k_knn_\w+<\d+, \d+, false", r["Kernel_Name"]):
                    vals[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(vals.items()):
    print(f"{c:40s} {sum(v) / len(v):16.1f}  ({len(v)} launches) {k}")
