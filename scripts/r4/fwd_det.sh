#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for env in "X=1" "ZOO_C3=0" "ZOO_I2_PIPE=0" "ZOO_PW=0" "ZOO_IGEMM2=0"; do
  echo "== $env"
  env $env timeout -k 10 120 python -u scripts/r4/fwd_det.py 2>&1 | grep -v "INFO\|amdgpu.ids" || exit 3
done
