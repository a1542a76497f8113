set -e
S=analytics-zoo_amd/tools/conv_sweep.py
timeout -k 10 120 python -u $S --detail > gpurun_out/sweep_base.log 2>&1
for wg in 512 2048 4096; do ZOO_WGRAD_WG=$wg timeout -k 10 100 python -u $S --ops wgrad >> gpurun_out/sweep.log 2>&1; done
for mp in 256 1024 2048; do ZOO_WGRAD_MINPIX=$mp timeout -k 10 100 python -u $S --ops wgrad >> gpurun_out/sweep.log 2>&1; done
ZOO_IGEMM_BN=64 timeout -k 10 100 python -u $S --ops fwd,dgrad >> gpurun_out/sweep.log 2>&1
