#!/bin/bash
# Local wrapper: rebuild the in-tree libraries (they travel with the snapshot),
# then run one gpurun call.  usage: scripts/gpu.sh TIMEOUT 'command'
set -e
cd "$(dirname "$0")/.."
make -s -C pbrt-v3-light-portals_amd -j8 ARCH=gfx950
make -s -C oracle
exec /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
