"""Summarise rocprofv3 kernel_stats.csv files: tools/kstats.py DIR..."""
import csv, glob, sys
for d in sys.argv[1:]:
    for f in sorted(glob.glob(d.rstrip('/') + '/**/*kernel_stats.csv', recursive=True)):
        rows = [r for r in csv.DictReader(open(f)) if 'lvk::' in r['Name'] and 'fill' not in r['Name']]
        print(f.split('/')[-2], '  '.join(f"{r['Name'].split('(')[0].replace('lvk::', '').replace('void ', '')}"
                                         f"={float(r['AverageNs']) / 1000:.1f}us" for r in rows))
