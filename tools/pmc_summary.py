"""Mean per-dispatch value of every counter in a rocprofv3 counter_collection.csv, for kernels whose name contains
the given substring.  usage: python tools/pmc_summary.py CSV [KERNEL_SUBSTRING]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # dispatch -> counter -> value
    for r in csv.DictReader(open(path)):
        if want in r["Kernel_Name"]:
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        sys.exit("no dispatch of %r in %s" % (want, path))
    names = sorted({n for d in per.values() for n in d})
    print("kernel~%s dispatches %d" % (want, len(per)))
    for n in names:
        vals = [d[n] for d in per.values() if n in d]
        print("%-26s %16.0f" % (n, sum(vals) / len(vals)))


if __name__ == "__main__":
    main()
