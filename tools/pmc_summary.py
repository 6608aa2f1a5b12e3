"""Average rocprofv3 --pmc counters per kernel over the pass directories under a
root (each g*/ holds one counter group's counter_collection.csv)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root):
    acc = defaultdict(lambda: defaultdict(list))
    for path in sorted(glob.glob(os.path.join(root, "g*", "**", "*counter_collection.csv"),
                                 recursive=True)):
        with open(path) as f:
            per_dispatch = defaultdict(lambda: defaultdict(float))
            names = {}
            for row in csv.DictReader(f):
                d = row["Dispatch_Id"]
                names[d] = row["Kernel_Name"]
                per_dispatch[d][row["Counter_Name"]] += float(row["Counter_Value"])
            for d, ctrs in per_dispatch.items():
                for c, v in ctrs.items():
                    acc[names[d]][c].append(v)
    for k, ctrs in acc.items():
        if "smamd" not in k:
            continue
        short = k.replace("void ", "").replace("smamd::(anonymous namespace)::", "")
        short = short.split("(")[0][:90]
        print(short)
        for c in sorted(ctrs):
            v = ctrs[c]
            print(f"   {c:28s} {sum(v) / len(v):16.0f}   (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmck")
