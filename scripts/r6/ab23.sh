#!/bin/bash
# r6 run 23: PMC passes over the ConvLSTM3D fused step kernels (32^3, T = 4, one iteration)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > /tmp/avail.txt 2>&1
python3 - > /tmp/passes.txt <<'PY'
import re
txt = open("/tmp/avail.txt").read()
have = set(re.findall(r"\b([A-Z][A-Z0-9_]+)\b", txt))
want = [
  ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD"],
  ["SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_WR", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_ACTIVE_INST_LDS"],
  ["FETCH_SIZE", "TCC_HIT_sum", "TA_BUSY_avr", "TA_FLAT_READ_WAVEFRONTS_sum"],
  ["WRITE_SIZE", "TCC_MISS_sum", "TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum"],
]
for p in want:
    ok = [c for c in p if c in have or re.sub(r"_(sum|avr|min|max)$", "", c) in have]
    print(" ".join(ok))
PY
cat /tmp/passes.txt
i=0
while read -r P; do
  i=$((i+1))
  [ -z "$P" ] && continue
  rm -rf /tmp/pmc$i
  timeout -s KILL 120 rocprofv3 --pmc $P -d /tmp/pmc$i -o p --output-format csv -- python3 analytics-zoo_amd/tools/convlstm_bench.py --dims 3 --T 4 --modes fused --iters 1 > gpurun_out/r6/ab23_pmc$i.log 2>&1 || { echo "pass $i rc=$?"; exit 50; }
  F=$(find /tmp/pmc$i -name "*counter_collection.csv" | head -1)
  python3 scripts/r6/pmc_sum.py $F > gpurun_out/r6/ab23_pmc${i}_sum.txt 2>&1
  cut -c1-600 gpurun_out/r6/ab23_pmc${i}_sum.txt
done < /tmp/passes.txt
