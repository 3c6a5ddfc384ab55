#!/bin/bash
# Copy the fox capture (transforms.json + the JPEGs present) from the reference tree into
# data/fox so it travels to the GPU box with the gpurun snapshot. data/ is git-ignored: the images are
# inputs, not part of this repository's history.
set -e
SRC=${1:-/root/reference/data/nerf/fox}
DST=$(dirname "$0")/../data/fox
mkdir -p "$DST/images"
cp "$SRC/transforms.json" "$DST/"
cp "$SRC"/images/*.jpg "$DST/images/"
echo "staged $(ls "$DST/images" | wc -l) images into $DST"
