#!/bin/bash
# Same-box A/B of the slab weight-gradient split size (NRSE_SLAB_MAX_TILES) on the default bench.
set -o pipefail
mkdir -p gpurun_out
bash tools/ab_env.sh "-" "NRSE_SLAB_MAX_TILES=256" "NRSE_SLAB_MAX_TILES=192"
