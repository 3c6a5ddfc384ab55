#!/bin/bash
# Copy the SDF meshes (BASELINE config C5: armadillo; bunny) from the reference tree into data/sdf so
# they travel to the GPU box with the gpurun snapshot. data/ is git-ignored (inputs, not history).
set -e
SRC=${1:-/root/reference/data/sdf}
DST=$(dirname "$0")/../data/sdf
mkdir -p "$DST"
cp "$SRC"/*.obj "$DST/"
ls -la "$DST"
