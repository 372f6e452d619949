"""Print the average kernel durations of rocprofv3 --stats CSVs (one or more directories)."""
import csv
import glob
import sys

for d in sys.argv[1:]:
    for f in sorted(glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            print(f"{d:40s} {r['Name'][:48]:48s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e3:9.1f} us")
