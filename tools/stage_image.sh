#!/bin/bash
# Copy the image primitive's training image (BASELINE config C1: albert.exr) from the reference tree into
# data/image so it travels to the GPU box with the gpurun snapshot. data/ is git-ignored (inputs).
set -e
SRC=${1:-/root/reference/data/image}
DST=$(dirname "$0")/../data/image
mkdir -p "$DST"
cp "$SRC"/albert.exr "$DST/"
ls -la "$DST"
