#!/bin/bash
# Build the HBM streaming probe for gfx950 next to its source (the binary is
# not committed: run this, then e.g. gpurun -- tools/probe/stream_probe).
set -e
cd "$(dirname "$0")"
hipcc --offload-arch=gfx950 -O3 -o stream_probe stream_probe.hip
# The decode GEMV probes (gemv5_probe.hip timing / PROBE_STAMPS timelines,
# xm_check.hip random-input correctness) include lowbit_gemv5.cuh directly.
# Build them like the library (xm_check runs each XM form against the generic
# kernel on random inputs):
#   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -DILLM_GEMV5_XM_IMPL -o xm_check xm_check.hip
# (-DILLM_GEMV5_XM_IMPL: define the XM launcher in the probe itself, as gemv_int4_xm.hip does)
