"""Per-kernel counter means from rocprofv3 --pmc counter_collection CSVs.

usage: pmc_summary.py FILTER CSV [CSV ...]
  FILTER: substring of the kernel names to keep (e.g. gemm8p)
Prints, per kernel name, every counter's mean value per dispatch."""
import csv
import sys
from collections import defaultdict


def main():
    filt, files = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(list))
    for f in files:
        per = defaultdict(float)
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if filt not in r["Kernel_Name"]:
                    continue
                per[(r["Kernel_Name"][:110], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, d, c), v in per.items():
            acc[k][c].append(v)
    for k, cs in acc.items():
        print(k)
        for c, vs in sorted(cs.items()):
            print(f"  {c:28s} {sum(vs) / len(vs):16.1f}   (n={len(vs)})")


if __name__ == "__main__":
    main()
