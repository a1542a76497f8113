#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for cfg in "80 0.05 32 0.5" "80 0.01 32 0.5" "200 0.02 32 0.5" "150 0.05 64 0.3" "300 0.01 32 0.5"; do
  timeout -k 10 200 python -u scripts/r4/dbg_fail.py train $cfg 2>&1 | grep "acc" || exit 3
done
