#!/bin/bash
# Cluster-sort A/B (tools/gpu_r3_csort.sh), then the dedisperser setup timing
# and the peak-heavy kernel trace (tools/gpu_r3_sig.sh).
set -o pipefail
./tools/gpu_r3_csort.sh && ./tools/gpu_r3_sig.sh
