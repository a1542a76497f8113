#!/bin/bash
# ResNet-50 default-knob sweep with the round-4 two-stream backward
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for env in "X=1" "ZOO_I2_BAND=0" "ZOO_C3=0" "ZOO_PW=0" "ZOO_WGRAD256_CONV_COUT=128" "ZOO_OPTIM_IN_BWD=0" "X=1" "ZOO_I2_BAND=0"; do
  v=$(env $env timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 2>&1 | grep -o '"value": [0-9.]*')
  echo "$env $v"
done
