#!/bin/bash
# ResNet-50 sweep of the conv-wgrad split target and the 224-row tile, band tiles off (default)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for env in "X=1" "ZOO_WGRAD256_CONV_WG=96" "ZOO_WGRAD256_CONV_WG=160" "ZOO_WGRAD256_CONV_WG=192" "ZOO_I2_Q224=0" "X=1" "ZOO_WGRAD256_CONV_WG=96" "ZOO_WGRAD256_CONV_WG=160"; do
  v=$(env $env timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 2>&1 | grep -o '"value": [0-9.]*') || exit 1
  echo "$env $v"
done
