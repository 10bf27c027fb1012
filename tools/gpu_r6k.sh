#!/bin/bash
# round 6: decode GEMV timing, production geometry: a = vgpr-form flag + generic only,
# b = no flag + XM forms, c = no flag + generic only, d = flag + XM forms (miscompiled)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
: > gpurun_out/r6k.jsonl
for rep in 1 2; do
  for v in a b c d; do
    PROBE_MODE=a timeout -k 10 120 tools/probe/gp_$v > gpurun_out/r6k_tmp.log 2>&1 || { tail -5 gpurun_out/r6k_tmp.log; exit 2; }
    sed "s/^{/{\"var\":\"$v\",\"rep\":$rep,/" gpurun_out/r6k_tmp.log >> gpurun_out/r6k.jsonl
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r6k.jsonl"):
    r = json.loads(l)
    if "us" in r: d[(r["op"], r["M"], r["normin"], r["var"])].append(r["us"])
    elif "check" in r and r["mismatch"]: print("CHECK FAIL", r)
keys = sorted({k[:3] for k in d})
print("op M normin | a(flag,gen) b(noflag,XM) c(noflag,gen) d(flag,XM)")
for k in keys:
    print(k, " ".join("%.2f" % min(d.get(k + (v,), [0])) for v in "abcd"))
PY
