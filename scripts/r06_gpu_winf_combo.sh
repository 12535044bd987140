#!/bin/bash
# Round 6: the hand-off split windows' probe modes, then the bands below 369.
set -o pipefail
./scripts/r06_gpu_winf_modes.sh && ./scripts/r06_gpu_winf_bands.sh
