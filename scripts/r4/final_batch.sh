#!/bin/bash
# end-of-round batch: 224x256 tile A/B, then the full GPU suite + smoke + bench, then profiles
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/r4/q224_ab.sh || exit 1
bash scripts/r4/gpu_full.sh full3 || exit 2
bash scripts/r4/prof_both.sh || exit 3
