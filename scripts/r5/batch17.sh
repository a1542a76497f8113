#!/bin/bash
# r5 batch 17: ConvLSTM step kernels in isolation (kernel trace + one counter pass)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_convlstm_seq.py \
  tests/test_gpu_keras_native.py -k "ConvLSTM or convlstm" > gpurun_out/r5/b17_cl_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r5/b17_cl_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u analytics-zoo_amd/tools/convlstm_bench.py > gpurun_out/r5/b17_convlstm_bench.log 2>&1 || exit 3
tail -1 gpurun_out/r5/b17_convlstm_bench.log

timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/prof_cs -o cs -- python3 analytics-zoo_amd/tools/convlstm_step_bench.py > gpurun_out/r5/b17_cs.log 2>&1 || exit 2
DB=$(find /tmp/prof_cs -name "*.db" | head -1)
python3 analytics-zoo_amd/tools/prof_summary.py $DB 1 "ConvLSTM step kernels" > gpurun_out/r5/b17_cs_summary.md 2>&1
grep -E "convlstm" gpurun_out/r5/b17_cs_summary.md
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_INSTS_MFMA -d /tmp/prof_cs2 -o cs2 -- python3 analytics-zoo_amd/tools/convlstm_step_bench.py --iters 2 > gpurun_out/r5/b17_pmc.log 2>&1 || exit 3
find /tmp/prof_cs2 -name "*counter_collection.csv" -exec cp {} gpurun_out/r5/b17_pmc.csv \;
ls -la gpurun_out/r5/b17_pmc.csv
ZOO_I2_KMIN=128 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_resnet50_parity.py tests/test_gpu_kernels.py -k "resnet" > gpurun_out/r5/b17_kmin_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r5/b17_kmin_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python -u bench.py > gpurun_out/r5/b17_def_$i.log 2>&1 || exit 20
  ZOO_I2_KMIN=128 timeout -k 10 200 python -u bench.py > gpurun_out/r5/b17_kmin_$i.log 2>&1 || exit 21
done
for f in gpurun_out/r5/b17_{def,kmin}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
