#!/bin/bash
# Round-4 first session: the default bench line (distinct in-flight buffers, serial k_link
# pricing), the counter list, and k_link's read requests split by size.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/r04a_bench.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 -L > $O/r04a_counters.txt 2>&1
P="bench.py --pmc-probe --config c2"
for c in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_BUBBLE_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  n=$(echo $c | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc $c -d $O/r04a_pmc_$n -o run --output-format csv -- python3 $P > $O/r04a_pmc_$n.log 2>&1
  echo "pmc $c rc $?" >> $O/r04a_pmc.log
done
exit 0
