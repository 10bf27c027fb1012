#!/bin/bash
# round-4: same-box A/B of the in-place grouped gxa slices (QLoRA), alternated
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
for i in 1 2; do
  $T 300 python -u tools/bench_qlora.py --steps 8 --warmup 2 > gpurun_out/qlora_ab_slices_$i.json 2>&1 || exit $?
  ILLM_LORA_GXA_SLICES=0 $T 300 python -u tools/bench_qlora.py --steps 8 --warmup 2 > gpurun_out/qlora_ab_cat_$i.json 2>&1 || exit $?
done
for f in gpurun_out/qlora_ab_*.json; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
