"""Per-kernel mean of every counter in rocprofv3 counter_collection CSVs.
usage: pmc_table.py DIR [DIR ...]"""
import csv, glob, os, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, '**', '*_counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('dsce::', '')
            if 'k_band' in r['Kernel_Name']:
                k = 'k_band<' + r['Kernel_Name'].split('<')[1].split(',')[0].replace('dsce::', '') + '>'
            acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
cols = sorted({c for v in acc.values() for c in v})
print('kernel'.ljust(28) + ''.join(c[:18].rjust(19) for c in cols))
for k, v in sorted(acc.items()):
    print(k[:27].ljust(28) + ''.join(('%.4g' % (sum(v[c]) / len(v[c])) if c in v else '-').rjust(19) for c in cols))
