#!/usr/bin/env python3
"""Summarise rocprofv3 counter CSVs: per kernel, the median value per dispatch of each counter."""
import collections
import csv
import glob
import statistics
import sys

d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
for f in sorted(glob.glob(d + '/p*/run_counter_collection.csv')):
    for row in csv.DictReader(open(f)):
        # (keyed by pass file and dispatch: a counter in two passes is two sets of dispatches, not one
        # summed set — round 4's stall summaries doubled SQ_WAVES that way)
        agg[row['Kernel_Name'][:48]][row['Counter_Name']][(f, int(row['Dispatch_Id']))] += float(row['Counter_Value'])
for kn, cs in agg.items():
    if 'skq' not in kn:
        continue
    print(kn)
    for c, per in sorted(cs.items()):
        v = sorted(per.values())
        print('   %-32s median %.4g  (n=%d, min %.4g, max %.4g)' % (c, statistics.median(v), len(v), v[0], v[-1]))
