#!/usr/bin/env python3
"""Sum the render kernel's PMC counters over a pmc_diag.sh output dir (one launch per pass)."""
import collections, csv, glob, sys
for d in sorted(glob.glob(sys.argv[1] + '/p*')):
    for f in glob.glob(d + '/**/run_counter_collection.csv', recursive=True):
        agg = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if 'render_unidir' in r['Kernel_Name']:
                agg[r['Counter_Name']] += float(r['Counter_Value'])
        for k, v in agg.items():
            print('%-40s %.5g' % (k, v))
