#!/bin/bash
# wgrad routing A/B: wgrad256 for the large-M stage-1 1x1 shapes and the 64/128-Cout 3x3 convs
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/wr; mkdir -p $O
run() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python -u analytics-zoo_amd/tools/conv_sweep.py --ops wgrad --detail > $O/$tag.log 2>&1 || return 1
  echo "$tag $(tail -1 $O/$tag.log)"
}
run base || exit 2
run mmax ZOO_WGRAD256_MMAX=1048576 || exit 3
run mmax_c64 ZOO_WGRAD256_MMAX=1048576 ZOO_WGRAD256_CMIN=64 || exit 4
run cout128 ZOO_WGRAD256_CONV_COUT=128 || exit 5
run cout64 ZOO_WGRAD256_CONV_COUT=64 || exit 6
python3 - <<'PY'
import json
rows = {}
for tag in ["base", "mmax", "mmax_c64", "cout128", "cout64"]:
    for l in open(f"gpurun_out/wr/{tag}.log"):
        if l.startswith('{"shape"'):
            r = json.loads(l); rows.setdefault(tuple(r["shape"]), {})[tag] = r["wgrad"]
for k, v in rows.items():
    print(k, " ".join(f"{t}={v.get(t, 0):.3f}" for t in ["base", "mmax", "mmax_c64", "cout128", "cout64"]))
PY
