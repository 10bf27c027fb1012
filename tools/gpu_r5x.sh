#!/bin/bash
# round 5: decode with the reordered v3 attention (_C.so) vs the previous attention (_C_attn0.so),
# then kernel traces of the current decode at B = 8 / 1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
: > gpurun_out/r5x_ab.jsonl
run() {  # B, lib
  IPEX_LLM_AMD_LIB=$2 BENCH_BATCH=$1 timeout -k 10 200 python bench.py --steps 64 --warmup 8 --no-tp-side > gpurun_out/r5x_tmp.log 2>&1 || { tail -5 gpurun_out/r5x_tmp.log; return 1; }
  tail -1 gpurun_out/r5x_tmp.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'B': $1, 'lib': '$2', 'tok_s': d['value'], 'ms': d['ms_per_step']}))" | tee -a gpurun_out/r5x_ab.jsonl
}
for i in 1 2; do
  for lib in _C.so _C_attn0.so; do run 1 $lib || exit 3; done
done
for lib in _C.so _C_attn0.so; do run 8 $lib || exit 3; done
for B in 8 1; do
  BENCH_BATCH=$B timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_x$B" -o run -- python3 "$R/bench.py" --steps 32 --warmup 4 --no-tp-side > "$R/gpurun_out/r5x_prof$B.log" 2>&1 || exit 5
  db=$(find gpurun_out/prof_x$B -name "*.db" | head -1)
  python3 tools/decode_trace_summary.py "$db" 5 > gpurun_out/r5x_trace_b$B.txt 2>&1 || exit 6
  rm -rf gpurun_out/prof_x$B
done
cat gpurun_out/r5x_trace_b8.txt | head -12
