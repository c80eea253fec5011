#!/bin/bash
# A/B of in-tree library variants (tdmpc_amd/libtdmpc_hip_<v>.so) on the literal single-env plan(): 6 alternating
# rounds of 150 calls per variant on one box, then the median per variant (the per-round spread is ~3 %)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=$(mktemp)
for i in 1 2 3 4 5 6; do
  for v in "$@"; do
    TDMPC_LIB_PATH=$PWD/tdmpc_amd/libtdmpc_hip_$v.so timeout -k 10 120 python -u tools/single_time.py humanoid-run 150 2>&1 | grep -v amdgpu.ids | sed "s/^/$v: /" | tee -a $out || exit 1
  done
done
python3 - "$out" <<'PY'
import re, statistics, sys, collections
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    m = re.match(r"(\S+): plan\(\) single env: ([0-9.]+) ms", line)
    if m: d[m.group(1)].append(float(m.group(2)))
for v, xs in d.items():
    print(f"{v}: median {statistics.median(xs):.4f} ms/call ({1e3 / statistics.median(xs):.1f} plan-steps/s), min {min(xs):.4f}, n={len(xs)}")
PY
