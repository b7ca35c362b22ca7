"""Print a rocprofv3 kernel_stats.csv compactly: name (80 chars), calls, average us, share."""
import csv
import sys

for r in list(csv.DictReader(open(sys.argv[1])))[:12]:
    print("%-80s %6s %10.2f us %6.2f%%" % (r["Name"][:80], r["Calls"], float(r["AverageNs"]) / 1e3,
                                          float(r.get("Percentage", 0) or 0)))
