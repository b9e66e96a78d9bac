#!/bin/bash
# rocprofv3 kernel stats of tools/pmc_probe.py; usage: tools/kstats.sh TAG [VAR=VAL ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
for kv in "$@"; do export "$kv"; done
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/ks_$tag" -- python3 tools/pmc_probe.py > gpurun_out/ks_$tag.log 2>&1 || exit 1
python3 - "$tag" <<'PY'
import csv, glob, sys
f = sorted(glob.glob('gpurun_out/ks_%s/**/*_kernel_stats.csv' % sys.argv[1], recursive=True))[-1]
for r in csv.DictReader(open(f)):
    n = r['Name'].replace('dsce::', '').replace('void ', '')
    n = n[:n.index('(')] if '(' in n else n
    print('%-60s %5s %10.1f us %6.2f%%' % (n[:60], r['Calls'], float(r['AverageNs']) / 1e3, float(r['Percentage'])))
PY
