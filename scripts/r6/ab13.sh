#!/bin/bash
# r6 run 13: NCF step trace (graph replay) and repeats
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2 3; do
  $T 300 python -u bench.py --model ncf --steps 200 --warmup 20 > gpurun_out/r6/ab13_ncf_$i.log 2>&1 || exit 21
  tail -1 gpurun_out/r6/ab13_ncf_$i.log | cut -c1-160
done
rm -rf /tmp/prof_ncf
$T 300 rocprofv3 --kernel-trace -d /tmp/prof_ncf -o ncf -- python3 bench.py --model ncf --steps 50 --warmup 10 > gpurun_out/r6/ab13_prof_ncf.log 2>&1 || exit 8
DB=$(find /tmp/prof_ncf -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_step.py $DB --totals > gpurun_out/r6/ab13_prof_ncf_totals.md 2>&1
head -24 gpurun_out/r6/ab13_prof_ncf_totals.md | cut -c1-160
python3 analytics-zoo_amd/tools/prof_step.py $DB ncf_fwd 3 --critical > gpurun_out/r6/ab13_prof_ncf_step.md 2>&1
tail -25 gpurun_out/r6/ab13_prof_ncf_step.md | cut -c1-160
