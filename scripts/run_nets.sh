set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_native_nets.py -q --timeout 200 --timeout-method thread > gpurun_out/pytest_nets.log 2>&1 || exit 1
$T 300 python analytics-zoo_amd/tools/zoo_models_bench.py --models mobilenet,mobilenet-v2,inception-v1,vgg-16,densenet-161,ssd300,ssd-mobilenet --batch 64 --steps 5 > gpurun_out/zoo_bench.log 2>&1 || exit 2
$T 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mbnet -o mb -- python3 analytics-zoo_amd/tools/zoo_models_bench.py --models mobilenet --mode infer --batch 64 --steps 10 > gpurun_out/prof_mbnet.log 2>&1 || exit 3
$T 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ssd -o ssd -- python3 analytics-zoo_amd/tools/zoo_models_bench.py --models ssd300 --batch 16 --steps 5 > gpurun_out/prof_ssd.log 2>&1 || exit 4
python analytics-zoo_amd/tools/prof_summary.py $(ls gpurun_out/prof_mbnet/*results.db | head -1) 13 "MobileNet v1 inference b64 (native NHWC)" > gpurun_out/prof_mbnet.md
python analytics-zoo_amd/tools/prof_summary.py $(ls gpurun_out/prof_ssd/*results.db | head -1) 7 "SSD-VGG16-300 training b16 (native NHWC)" > gpurun_out/prof_ssd.md
rm -rf gpurun_out/prof_mbnet gpurun_out/prof_ssd
