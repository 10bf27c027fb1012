#!/bin/bash
# round-4: prefill (first token) kernel time vs wall at B=1 and B=8
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for B in 1 8; do
  cd /tmp && export TMPDIR=/tmp
  BENCH_BATCH=$B timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_pf$B" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 > "$R/gpurun_out/prof_pf$B.log" 2>&1 || exit $?
  cd "$R"
  db=$(find gpurun_out/prof_pf$B -name "*.db" | head -1)
  python3 tools/prefill_window.py "$db" > gpurun_out/prefill_window_b$B.txt 2>&1
  cat gpurun_out/prefill_window_b$B.txt
  rm -rf gpurun_out/prof_pf$B
done
