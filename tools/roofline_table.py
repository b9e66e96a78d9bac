"""Per-kernel HBM roofline from a tools/pmc_session.sh directory: bytes per
launch = (2 FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 correction,
MI355X_MICROARCH.md §HBM), duration from the same passes' kernel traces.
usage: roofline_table.py gpurun_out/pmc_TAG [peak_GBps]"""
import collections, csv, glob, os, sys

d = sys.argv[1]
peak = float(sys.argv[2]) if len(sys.argv) > 2 else 8000.0


def key(name):
    n = name.replace('void ', '').replace('dsce::', '')
    if n.startswith('k_band'):
        return 'k_band<' + n.split('<')[1].split(',')[0].split('(')[0] + '>'
    return n.split('(')[0]


ctr = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in glob.glob(os.path.join(d, '**', '*_counter_collection.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
        ctr[key(r['Kernel_Name'])][r['Counter_Name']].append(float(r['Counter_Value']))
for f in glob.glob(os.path.join(d, '**', '*_kernel_trace.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
        dur[key(r['Kernel_Name'])].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9)
print('%-34s %9s %10s %9s %6s' % ('kernel', 'us/launch', 'HBM MB', 'GB/s', 'frac'))
for k in sorted(ctr, key=lambda k: -sum(dur.get(k, [0]))):
    c = ctr[k]
    if 'FETCH_SIZE' not in c or 'WRITE_SIZE' not in c or not dur.get(k):
        continue
    b = (2 * sum(c['FETCH_SIZE']) / len(c['FETCH_SIZE']) + sum(c['WRITE_SIZE']) / len(c['WRITE_SIZE'])) * 1024
    t = sum(dur[k]) / len(dur[k])
    if t * 1e6 < 20:
        continue
    print('%-34s %9.1f %10.1f %9.0f %6.2f' % (k[:34], t * 1e6, b / 1e6, b / t / 1e9, b / t / 1e9 / peak))
