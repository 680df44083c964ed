"""Average rocprofv3 --pmc counters per kernel (name substring) from the
counter_collection CSVs under a directory: pmc_sq.py DIR [substring]."""
import collections, csv, glob, os, sys

root, sub = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "gf_bs_kernel")
acc = collections.defaultdict(list)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if sub in row.get("Kernel_Name", ""):
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(acc):
    v = acc[k]
    print(f"{k:28s} n={len(v):4d} avg={sum(v) / len(v):16.1f}")
