#!/bin/bash
# Build the HBM streaming probe for gfx950 next to its source (the binary is
# not committed: run this, then e.g. gpurun -- tools/probe/stream_probe).
set -e
cd "$(dirname "$0")"
hipcc --offload-arch=gfx950 -O3 -o stream_probe stream_probe.hip
