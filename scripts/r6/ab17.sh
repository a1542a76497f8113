#!/bin/bash
# r6 run 17: shortcut dgrad prologue on the plain-epilogue pw kernel, y2 only where pw takes it; tests, bench x3,
# fresh ResNet-50 step trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_shortcut_bn.py tests/test_gpu_resnet50_parity.py tests/test_gpu_pw.py tests/test_gpu_bnfold.py tests/test_gpu_fwd_pro.py -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r6/ab17_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6/ab17_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2 3; do
  $T 300 python -u bench.py > gpurun_out/r6/ab17_fs_$i.log 2>&1 || exit 22
  python3 -c "import json; d=json.loads(open('gpurun_out/r6/ab17_fs_$i.log').read().strip().splitlines()[-1]); print('fs', d['value'], d['ms_per_step'], d['first_loss'], d['final_loss'])"
done
rm -rf /tmp/prof_rn
$T 300 rocprofv3 --kernel-trace -d /tmp/prof_rn -o rn -- python3 bench.py --input device --steps 8 --warmup 3 > gpurun_out/r6/ab17_prof_rn.log 2>&1 || exit 8
DB=$(find /tmp/prof_rn -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_step.py $DB --critical > gpurun_out/r6/ab17_prof_rn_step.md 2>&1
grep -A30 "^## Critical" gpurun_out/r6/ab17_prof_rn_step.md | head -24
tail -2 gpurun_out/r6/ab17_prof_rn_step.md
