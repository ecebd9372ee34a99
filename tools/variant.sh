#!/bin/bash
# Build an experimental variant of the HIP library into build/<name>/ (CPU side):
#   tools/variant.sh NAME [extra hipcc flags...]
# then on the GPU box: GFPL_LIB_DIR=build/NAME python bench.py ...  (tools/ab.sh)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p build/$name
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared -Wall -Wno-unused-result \
    -Iinclude "$@" gf-pl-slam_amd/csrc/*.hip gf-pl-slam_amd/csrc/*.cpp -o build/$name/libgfpl_hip.so
cp gf-pl-slam_amd/lib/libgfpl_synth.so build/$name/
echo "built build/$name"
