"""Per-kernel table of a rocprofv3 --stats kernel_stats.csv."""
import csv
import sys

for path in sys.argv[1:]:
    print("==", path)
    for r in csv.DictReader(open(path)):
        n = r["Name"].split("(")[0][:60]
        print("%-60s %5s calls  avg %9.1f us  total %8.2f ms" % (
            n, r["Calls"], float(r["AverageNs"]) / 1e3,
            float(r["TotalDurationNs"]) / 1e6))
