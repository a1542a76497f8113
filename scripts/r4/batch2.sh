#!/bin/bash
# round-4 validation batch 2: per-conv roofline, ResNet profile, NCF bench + profile, wgrad split A/B, int8/fp8
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/b2; mkdir -p $O
timeout -k 10 240 python -u analytics-zoo_amd/tools/conv_sweep.py --detail --roofline $O/resnet50_roofline.md > $O/conv_sweep.log 2>&1 || exit 2
tail -1 $O/conv_sweep.log
bash scripts/r4/prof_resnet.sh c3 > $O/prof_rn.out 2>&1 || exit 3
head -24 gpurun_out/prof_rn_c3_summary.md
timeout -k 10 200 python -u bench.py --model ncf --batch 65536 --steps 50 --warmup 10 > $O/bench_ncf.log 2>&1 || exit 4
echo "ncf $(tail -1 $O/bench_ncf.log)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_ncf -o ncf -- python3 bench.py --model ncf --batch 65536 --steps 32 --warmup 10 > $O/prof_ncf.log 2>&1 || exit 5
DB=$(find /tmp/prof_ncf -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_summary.py $DB 42 "NCF ml-20m shape b65536 (bench.py --model ncf under rocprofv3), round 4" > $O/ncf_prof.md 2>&1
head -16 $O/ncf_prof.md
for wg in 256 128 64; do
  ZOO_WGRAD256_WG=$wg timeout -k 10 200 python -u analytics-zoo_amd/tools/conv_sweep.py --ops wgrad > $O/wg_rn_$wg.log 2>&1 || exit 6
  echo "WG=$wg resnet $(tail -1 $O/wg_rn_$wg.log)"
  ZOO_WGRAD256_WG=$wg timeout -k 10 200 python -u analytics-zoo_amd/tools/wgrad_bench.py > $O/wg_bert_$wg.log 2>&1 || exit 7
  python3 -c "
import json
for l in open('$O/wg_bert_$wg.log'):
    if l.startswith('{'):
        r=json.loads(l); print('  bert', r['M'], r['N'], r['K'], r['zoo_wgrad256']['us'], 'us')
"
done
timeout -k 10 400 python -u analytics-zoo_amd/tools/quant_bench.py --batch 256 --iters 20 > $O/quant.log 2>&1 || exit 8
tail -6 $O/quant.log
