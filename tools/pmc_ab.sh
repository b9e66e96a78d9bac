#!/bin/bash
# Counter passes of the in-tree library vs ab/libdsce_alt.so over tools/pmc_probe.py
# (run via gpurun from the repo root): tools/pmc_ab.sh TAG KERNEL_REGEX "CTRS1" ["CTRS2" ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift; kre=$1; shift
lib=channel-estimation_amd/dsce/libdsce.so
cp $lib /tmp/libdsce_base.so || exit 1
export TMPDIR=/tmp
for v in base alt; do
  if [ $v = base ]; then cp /tmp/libdsce_base.so $lib; else cp ab/libdsce_alt.so $lib; fi
  i=0
  for ctr in "$@"; do
    d=gpurun_out/pmcab_${tag}_${v}_$i
    timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$d" -- python3 tools/pmc_probe.py 65536 > $d.log 2>&1 || { echo "pass $v $i failed"; tail -5 $d.log; cp /tmp/libdsce_base.so $lib; exit 1; }
    echo "== $v pass $i"; python3 tools/pmc_table.py $d | cut -c1-260 | grep -E "kernel|$kre"
    i=$((i + 1))
  done
done
cp /tmp/libdsce_base.so $lib
echo all_ok
