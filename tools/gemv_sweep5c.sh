#!/bin/bash
# GLU workgroup-size sweep (GPU box): gpurun_out/sweep5c.log
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/sweep5c.log
timeout -k 10 120 python tools/gemv_sweep5.py 1,2,4,8,16 >> gpurun_out/sweep5c.log 2>&1 || exit $?
for cfg in "8 1" "8 2" "8 4" "4 1" "4 2"; do set -- $cfg
  ILLM_GEMV5_NW=$1 ILLM_GEMV5_KW=$2 timeout -k 10 120 python tools/gemv_sweep5.py 2,4,8,16 glu | sed "s/\"kw\"/\"nw\": $1, \"kw\"/" >> gpurun_out/sweep5c.log 2>&1 || exit $?
done
for cfg in "8 1" "8 2"; do set -- $cfg
  ILLM_GEMV5_NW=$1 ILLM_GEMV5_KW=$2 timeout -k 10 120 python tools/gemv_sweep5.py 1,8,16 qkv,o,down | sed "s/\"kw\"/\"nw\": $1, \"kw\"/" >> gpurun_out/sweep5c.log 2>&1 || exit $?
done
grep -c us gpurun_out/sweep5c.log
